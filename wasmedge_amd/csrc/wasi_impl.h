// wasi_impl.h -- the built-in WASI subset (wasi_snapshot_preview1) served on the host
// for lanes that yield at a WASI import. One restatement, two users: the product
// library (wasi.cpp, memory through the host-call round's wave view) and the test
// emulator (emu.cpp, contiguous memory). Semantics follow the reference's host functions
// (lib/host/wasi/wasifunc.cpp) over its Environ / VINode / INode (include/host/wasi/
// environ.h, vinode.h, lib/host/wasi/vinode.cpp, inode-linux.cpp), with the default stdio
// rights (lib/host/wasi/environ.cpp:38-46):
//   args_get / args_sizes_get      wasifunc.cpp:314-372, environ.h:85-114
//   environ_get / environ_sizes_get wasifunc.cpp:374-433, environ.h:127-157
//   fd_write                       wasifunc.cpp:990-1046; fds 1/2 are captured per
//                                  instance; stdin has no write right (NOTCAPABLE,
//                                  vinode.h:337-343); a directory or a file opened for
//                                  reading: BADF (writev on an O_RDONLY fd)
//   proc_exit                      wasifunc.cpp:1550-1554 (exit code, then Terminated)
//   sched_yield                    wasifunc.cpp:1571-1576
//   fd_prestat_get / _dir_name     wasifunc.cpp:724-766, environ.h:385-420: BADF for an fd
//                                  with no node, INVAL for a node with no name (stdio,
//                                  opened files), else tag DIR and the preopen's name
//   path_open                      wasifunc.cpp:1198-1268, environ.h:693-710,
//                                  vinode.cpp:190-234 (rights), resolvePath :385-523
//   fd_read / fd_seek / fd_tell    wasifunc.cpp:828-882, 927-988, vinode.h:252-327
//   fd_close                       wasifunc.cpp:525-533, environ.h:230-241 (preopens NOTSUP)
//   fd_fdstat_get / _set_flags     wasifunc.cpp:545-581, vinode.h:116-145, inode-linux.cpp:206
//   fd_filestat_get                wasifunc.cpp:611-630, inode-linux.cpp:261-276
//   path_filestat_get              wasifunc.cpp:1072-1108, vinode.cpp:127-141
//   clock_time_get / clock_res_get wasifunc.cpp:434-489 (the pointer first, then the id)
//   random_get                     wasifunc.cpp:1578-1596, environ.h:834-850
// Preopened directories ("guest:host", WasmEdge_BatchInitWASIWithPreopens) bind with the
// reference's rights (kReadRights | kWriteRights | kCreateRights, environ.cpp:17-71) and
// behave as a READ-ONLY mount, since N instances share one host directory: an open that
// would create, truncate or write fails with ROFS as open(2) does there. A file is read
// whole when a lane opens it and keeps those bytes and that stat (a snapshot shared by the
// lanes). Where the reference is random -- the numbers of new fds (environ.h:1096-1108)
// and random_get -- a per-lane splitmix64 draws them (seeded at InitWASI from the host's
// random device, or by WasmEdge_BatchWASISetDeterministic, which also fixes the clocks to
// a start time advancing 1 us per call); stdin reads end-of-file; stdout/stderr are the
// per-instance captures, and their fdstat/filestat describe a character device (the
// reference fstat()s the host process's own fds 0-2).
// Args may be given per instance (WasmEdge_BatchWASISetInstanceArgs); the reference builds
// one Environ per VM, so per-instance args are per-VM args.
// Every pointer is bounds-checked like MemoryInstance::getPointer (memory.h:226-233:
// Offset + sizeof(T) * Count <= size, the product in 32 bits) before anything is written.
#pragma once
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

namespace wbw {

enum : uint32_t {                       // thirdparty/wasi/api.hpp
  ERRNO_SUCCESS = 0, ERRNO_ACCES = 2, ERRNO_BADF = 8, ERRNO_EXIST = 20, ERRNO_FAULT = 21,
  ERRNO_INVAL = 28, ERRNO_ISDIR = 31, ERRNO_LOOP = 32, ERRNO_NOENT = 44, ERRNO_NOTDIR = 54,
  ERRNO_NOTSUP = 58, ERRNO_ROFS = 69, ERRNO_SPIPE = 70, ERRNO_NOTCAPABLE = 76
};
enum : uint8_t { FILETYPE_UNKNOWN = 0, FILETYPE_CHARACTER_DEVICE = 2, FILETYPE_DIRECTORY = 3,
                 FILETYPE_REGULAR_FILE = 4, FILETYPE_SYMBOLIC_LINK = 7 };
// __wasi_rights_t bits
namespace rights {
constexpr uint64_t FD_DATASYNC = 1ull << 0, FD_READ = 1ull << 1, FD_SEEK = 1ull << 2,
                   FD_FDSTAT_SET_FLAGS = 1ull << 3, FD_SYNC = 1ull << 4, FD_TELL = 1ull << 5,
                   FD_WRITE = 1ull << 6, FD_ADVISE = 1ull << 7, FD_ALLOCATE = 1ull << 8,
                   PATH_CREATE_DIRECTORY = 1ull << 9, PATH_CREATE_FILE = 1ull << 10,
                   PATH_LINK_SOURCE = 1ull << 11, PATH_LINK_TARGET = 1ull << 12,
                   PATH_OPEN = 1ull << 13, FD_READDIR = 1ull << 14, PATH_READLINK = 1ull << 15,
                   PATH_RENAME_SOURCE = 1ull << 16, PATH_RENAME_TARGET = 1ull << 17,
                   PATH_FILESTAT_GET = 1ull << 18, PATH_FILESTAT_SET_SIZE = 1ull << 19,
                   PATH_FILESTAT_SET_TIMES = 1ull << 20, FD_FILESTAT_GET = 1ull << 21,
                   FD_FILESTAT_SET_SIZE = 1ull << 22, FD_FILESTAT_SET_TIMES = 1ull << 23,
                   PATH_SYMLINK = 1ull << 24, PATH_REMOVE_DIRECTORY = 1ull << 25,
                   PATH_UNLINK_FILE = 1ull << 26, POLL_FD_READWRITE = 1ull << 27,
                   SOCK_SHUTDOWN = 1ull << 28, ALL = (1ull << 36) - 1;   // (cast<__wasi_rights_t>)
// lib/host/wasi/environ.cpp:17-46
constexpr uint64_t READ = FD_ADVISE | FD_FILESTAT_GET | FD_READ | FD_READDIR | FD_SEEK | FD_TELL |
                          PATH_FILESTAT_GET | PATH_LINK_SOURCE | PATH_OPEN | PATH_READLINK |
                          PATH_RENAME_SOURCE | POLL_FD_READWRITE | SOCK_SHUTDOWN;
constexpr uint64_t WRITE = FD_ADVISE | FD_ALLOCATE | FD_DATASYNC | FD_FDSTAT_SET_FLAGS |
                           FD_FILESTAT_SET_SIZE | FD_FILESTAT_SET_TIMES | FD_SYNC | FD_WRITE |
                           PATH_FILESTAT_SET_SIZE | PATH_FILESTAT_SET_TIMES | PATH_OPEN |
                           PATH_REMOVE_DIRECTORY | PATH_RENAME_TARGET | PATH_UNLINK_FILE |
                           POLL_FD_READWRITE | SOCK_SHUTDOWN;
constexpr uint64_t CREATE = PATH_CREATE_DIRECTORY | PATH_CREATE_FILE | PATH_LINK_TARGET |
                            PATH_OPEN | PATH_RENAME_TARGET | PATH_SYMLINK;
constexpr uint64_t STDIN = FD_ADVISE | FD_FILESTAT_GET | FD_READ | POLL_FD_READWRITE;
constexpr uint64_t STDOUT = FD_ADVISE | FD_DATASYNC | FD_FILESTAT_GET | FD_SYNC | FD_WRITE |
                            POLL_FD_READWRITE;
}  // namespace rights
constexpr uint8_t kPreopenTypeDir = 0;  // __WASI_PREOPENTYPE_DIR
constexpr uint32_t kIOVMax = 1024;      // include/host/wasi/environ.h:33
constexpr uint32_t kMaxArgs = 9;        // operands of the widest function (path_open)
constexpr uint8_t kTerminated = 0x01;   // ErrCode::Terminated (enum.inc)
constexpr int kMaxNestedLinks = 8;      // vinode.cpp:23

enum Fn { ARGS_GET, ARGS_SIZES_GET, ENVIRON_GET, ENVIRON_SIZES_GET, FD_WRITE, PROC_EXIT,
          SCHED_YIELD, FD_PRESTAT_GET, FD_PRESTAT_DIR_NAME, PATH_OPEN, FD_READ, FD_SEEK, FD_TELL,
          FD_CLOSE, FD_FDSTAT_GET, FD_FDSTAT_SET_FLAGS, FD_FILESTAT_GET, PATH_FILESTAT_GET,
          CLOCK_TIME_GET, CLOCK_RES_GET, RANDOM_GET, NUM_FNS };

// a host file as a lane opened it: its bytes and its stat (shared by the lanes)
struct Blob {
  std::vector<uint8_t> bytes;
  struct stat st;
};

// configuration shared by every instance (WasmEdge_ImportObjectCreateWASI's Args/Envs/
// Preopens): preopens are the guest names of fds 3, 4, ... (environ.cpp:54-93), host the
// directories they stand for
struct Env {
  std::vector<std::string> args, envs, preopens, host;
  uint64_t seed = 0;              // the lanes' generators (fd numbers, random_get)
  bool fixed_clock = false;       // clocks: clock_ns + 1 us per call of the lane
  uint64_t clock_ns = 0;
  std::mutex mu;                  // (the blob cache: lanes are served on several threads)
  std::map<std::string, std::shared_ptr<const Blob>> blobs;
  // the file at `path`, read whole the first time any lane opens it; null + *err (errno)
  std::shared_ptr<const Blob> blob(const std::string &path, int *err) {
    std::lock_guard<std::mutex> g(mu);
    auto it = blobs.find(path);
    if (it != blobs.end()) return it->second;
    auto b = std::make_shared<Blob>();
    const int fd = ::open(path.c_str(), O_RDONLY | O_NOFOLLOW | O_CLOEXEC);
    if (fd < 0 || ::fstat(fd, &b->st) != 0) {
      *err = errno;
      if (fd >= 0) ::close(fd);
      return nullptr;
    }
    if (S_ISREG(b->st.st_mode)) {
      b->bytes.resize(size_t(b->st.st_size));
      size_t got = 0;
      while (got < b->bytes.size()) {
        const ssize_t r = ::read(fd, b->bytes.data() + got, b->bytes.size() - got);
        if (r <= 0) break;
        got += size_t(r);
      }
      b->bytes.resize(got);
    }
    ::close(fd);
    blobs[path] = b;
    return b;
  }
};

// one node of a lane's fd table (Environ::FdMap -> VINode)
struct Fd {
  enum Kind { STDIN, STDOUT, STDERR, DIR, FILE } kind = STDIN;
  int pre = -1;              // the preopen it is (-1: none; only preopens have a name)
  std::string host;          // directories and files: the host path
  uint32_t depth = 0;        // directories below its preopen (how far ".." may climb)
  uint64_t rb = 0, ri = 0;   // FsRightsBase / FsRightsInheriting
  std::shared_ptr<const Blob> blob;
  uint64_t off = 0;
};

// per-instance WASI state: captured stdout/stderr, the proc_exit code, the instance's own
// args when it has them, its fd table (built at its first fd call), its generator and
// clock
struct Lane {
  std::string out[2];
  uint32_t exit_code = 0;
  bool own_args = false;
  std::vector<std::string> args;
  uint32_t index = 0;              // the instance id (seeds the generator)
  bool fs_ready = false;
  std::map<uint32_t, Fd> fds;
  uint64_t rng = 0, clock_calls = 0;
};

// VINode::canonicalGuest (lib/host/wasi/vinode.cpp:54-97), the name a preopen binds under:
// leading slashes dropped, "." kept only as the first part, ".." pops, "" -> "/"
inline std::string canonical_guest(const std::string &path) {
  std::vector<std::string> parts;
  size_t i = 0;
  while (i < path.size() && path[i] == '/') i++;
  while (i < path.size()) {
    size_t j = path.find('/', i);
    if (j == std::string::npos) j = path.size();
    const std::string part = path.substr(i, j - i);
    while (j < path.size() && path[j] == '/') j++;
    if (part == "..") {
      if (!parts.empty()) parts.pop_back();
    } else if (part[0] != '.' || parts.size() != 1) {
      parts.push_back(part);
    }
    i = j;
  }
  if (parts.empty()) parts.push_back("");
  std::string r;
  for (const auto &p : parts) r += p + "/";
  r.pop_back();
  return r.empty() ? std::string("/") : r;
}

// "guest:host" or one path for both (environ.cpp:57-66): the guest name and the host
// directory (absolute when it exists)
inline void add_preopen(Env &env, const std::string &d) {
  const size_t colon = d.find(':');
  env.preopens.push_back(canonical_guest(colon == std::string::npos ? d : d.substr(0, colon)));
  const std::string h = colon == std::string::npos ? d : d.substr(colon + 1);
  char *rp = ::realpath(h.c_str(), nullptr);
  env.host.push_back(rp ? std::string(rp) : h);
  free(rp);
}
inline uint64_t host_seed() {
  std::random_device rd;
  return (uint64_t(rd()) << 32) | rd();
}

// one instance's linear memory
struct MemIO {
  virtual ~MemIO() {}
  virtual bool present() = 0;                     // the module has a memory
  virtual uint64_t size() = 0;                    // bytes (pages * 64 KiB)
  virtual bool read(uint32_t off, uint32_t len, uint8_t *dst) = 0;    // in bounds only
  virtual bool write(uint32_t off, uint32_t len, const uint8_t *src) = 0;
};

// The import `name` of module wasi_snapshot_preview1 with value types (0x7F i32, 0x7E i64)
// `params` -> `results`, or -1 if not in the subset / of another signature (then the import
// stays unbound and a lane reaching it reports 0xB1).
inline int lookup(const std::string &name, const std::vector<uint8_t> &params,
                  const std::vector<uint8_t> &results) {
  struct S { const char *n; Fn f; const char *p, *r; };   // 'i' i32, 'I' i64
  static const S tab[] = {{"args_get", ARGS_GET, "ii", "i"},
                          {"args_sizes_get", ARGS_SIZES_GET, "ii", "i"},
                          {"environ_get", ENVIRON_GET, "ii", "i"},
                          {"environ_sizes_get", ENVIRON_SIZES_GET, "ii", "i"},
                          {"fd_write", FD_WRITE, "iiii", "i"},
                          {"proc_exit", PROC_EXIT, "i", ""},
                          {"sched_yield", SCHED_YIELD, "", "i"},
                          {"fd_prestat_get", FD_PRESTAT_GET, "ii", "i"},
                          {"fd_prestat_dir_name", FD_PRESTAT_DIR_NAME, "iii", "i"},
                          {"path_open", PATH_OPEN, "iiiiiIIii", "i"},
                          {"fd_read", FD_READ, "iiii", "i"},
                          {"fd_seek", FD_SEEK, "iIii", "i"},
                          {"fd_tell", FD_TELL, "ii", "i"},
                          {"fd_close", FD_CLOSE, "i", "i"},
                          {"fd_fdstat_get", FD_FDSTAT_GET, "ii", "i"},
                          {"fd_fdstat_set_flags", FD_FDSTAT_SET_FLAGS, "ii", "i"},
                          {"fd_filestat_get", FD_FILESTAT_GET, "ii", "i"},
                          {"path_filestat_get", PATH_FILESTAT_GET, "iiiii", "i"},
                          {"clock_time_get", CLOCK_TIME_GET, "iIi", "i"},
                          {"clock_res_get", CLOCK_RES_GET, "ii", "i"},
                          {"random_get", RANDOM_GET, "ii", "i"}};
  auto vt = [](char c) { return uint8_t(c == 'I' ? 0x7E : 0x7F); };
  for (const S &s : tab) {
    if (name != s.n) continue;
    const std::string p = s.p, r = s.r;
    if (params.size() != p.size() || results.size() != r.size()) return -1;
    for (size_t k = 0; k < p.size(); k++) if (params[k] != vt(p[k])) return -1;
    for (size_t k = 0; k < r.size(); k++) if (results[k] != vt(r[k])) return -1;
    return s.f;
  }
  return -1;
}

inline bool in_bounds(MemIO &m, uint32_t off, uint32_t size, uint32_t count) {
  const uint32_t bytes = size * count;   // getPointer: uint32 ByteSize
  return uint64_t(off) + bytes <= m.size();
}
inline void put_le(MemIO &m, uint32_t off, uint64_t v, uint32_t n) {
  uint8_t b[8];
  for (uint32_t k = 0; k < n; k++) b[k] = uint8_t(v >> (8 * k));
  m.write(off, n, b);
}
inline void put_u32(MemIO &m, uint32_t off, uint32_t v) { put_le(m, off, v, 4); }
inline uint32_t get_u32(MemIO &m, uint32_t off) {
  uint8_t b[4] = {0, 0, 0, 0};
  m.read(off, 4, b);
  return uint32_t(b[0]) | uint32_t(b[1]) << 8 | uint32_t(b[2]) << 16 | uint32_t(b[3]) << 24;
}

inline uint32_t buffer_size(const std::vector<std::string> &v) {   // calculateBufferSize
  uint32_t s = 0;
  for (const auto &x : v) s += uint32_t(x.size()) + 1;
  return s;
}

// args_get / environ_get: pointers [n+1] (the last one 0), NUL-terminated strings
inline uint32_t list_get(MemIO &m, const std::vector<std::string> &v, uint32_t ptrs, uint32_t buf) {
  if (!m.present()) return ERRNO_FAULT;
  const uint32_t count = uint32_t(v.size()) + 1, bsize = buffer_size(v);
  if (!in_bounds(m, ptrs, 4, count)) return ERRNO_FAULT;
  if (!in_bounds(m, buf, 1, bsize)) return ERRNO_FAULT;
  // the reference's write order (the two areas may overlap): Argv[0] = buf, then per
  // string its bytes and Argv[k+1] = Argv[k] + size (Argv[k] read back), then Argv[n] = 0
  put_u32(m, ptrs, buf);
  uint32_t p = buf;
  for (uint32_t k = 0; k < v.size(); k++) {
    const uint32_t size = uint32_t(v[k].size()) + 1;
    m.write(p, size, reinterpret_cast<const uint8_t *>(v[k].c_str()));
    p += size;
    put_u32(m, ptrs + 4 * (k + 1), get_u32(m, ptrs + 4 * k) + size);
  }
  put_u32(m, ptrs + 4 * uint32_t(v.size()), 0);
  return ERRNO_SUCCESS;
}

// args_sizes_get / environ_sizes_get: both pointers checked, then count, then size
inline uint32_t list_sizes(MemIO &m, const std::vector<std::string> &v, uint32_t pc, uint32_t ps) {
  if (!m.present()) return ERRNO_FAULT;
  if (!in_bounds(m, pc, 4, 1) || !in_bounds(m, ps, 4, 1)) return ERRNO_FAULT;
  put_u32(m, pc, uint32_t(v.size()));
  put_u32(m, ps, buffer_size(v));
  return ERRNO_SUCCESS;
}

// ---- the fd table
inline uint64_t next_rand(Lane &lane) {   // splitmix64
  uint64_t z = (lane.rng += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// Environ::init (environ.cpp:54-93): fds 0-2 the stdio nodes, 3.. the preopens
inline void fs_ready(const Env &env, Lane &lane) {
  if (lane.fs_ready) return;
  lane.fs_ready = true;
  lane.rng = env.seed + (uint64_t(lane.index) + 1) * 0xD1B54A32D192ED03ull;
  lane.fds[0].kind = Fd::STDIN;
  lane.fds[0].rb = rights::STDIN;
  lane.fds[1].kind = Fd::STDOUT;
  lane.fds[1].rb = rights::STDOUT;
  lane.fds[2].kind = Fd::STDERR;
  lane.fds[2].rb = rights::STDOUT;
  for (size_t k = 0; k < env.preopens.size(); k++) {
    Fd &f = lane.fds[uint32_t(3 + k)];
    f.kind = Fd::DIR;
    f.pre = int(k);
    f.host = env.host[k];
    f.rb = f.ri = rights::READ | rights::WRITE | rights::CREATE;   // environ.cpp:67-71
  }
}
inline Fd *fd_of(const Env &env, Lane &lane, int32_t fd) {     // Environ::getNodeOrNull
  fs_ready(env, lane);
  auto it = lane.fds.find(uint32_t(fd));
  return it == lane.fds.end() ? nullptr : &it->second;
}
inline bool can(const Fd &f, uint64_t rb, uint64_t ri = 0) {   // VINode::can
  return (f.rb & rb) == rb && (f.ri & ri) == ri;
}
inline uint32_t from_errno(int e) {   // inode-linux fromErrNo, for the cases met here
  switch (e) {
    case ENOENT: return ERRNO_NOENT;
    case ENOTDIR: return ERRNO_NOTDIR;
    case ELOOP: return ERRNO_LOOP;
    case EISDIR: return ERRNO_ISDIR;
    case EINVAL: return ERRNO_INVAL;
    default: return ERRNO_ACCES;
  }
}
inline uint8_t filetype_of(mode_t m) {
  if (S_ISREG(m)) return FILETYPE_REGULAR_FILE;
  if (S_ISDIR(m)) return FILETYPE_DIRECTORY;
  if (S_ISLNK(m)) return FILETYPE_SYMBOLIC_LINK;
  if (S_ISCHR(m)) return FILETYPE_CHARACTER_DEVICE;
  return FILETYPE_UNKNOWN;
}
inline uint64_t ns_of(const struct timespec &t) { return uint64_t(t.tv_sec) * 1000000000ull + uint64_t(t.tv_nsec); }
inline int stat_of(const Fd &f, struct stat *st) {   // files as opened, directories now
  if (f.kind == Fd::FILE && f.blob) { *st = f.blob->st; return 0; }
  return ::stat(f.host.c_str(), st) == 0 ? 0 : errno;
}

// VINode::resolvePath (vinode.cpp:385-523) from directory node `d`: the host directory
// that holds the path's last part (*dir) and that part (*last, "." for the directory
// itself). ".." stops at the preopen (NOTCAPABLE); symbolic links inside the path are
// followed (at most kMaxNestedLinks), the last part only with SYMLINK_FOLLOW.
inline uint32_t resolve(const Fd &d, std::string path, uint32_t lookup, std::string *dir, std::string *last) {
  std::string cur = d.host, root = d.host;
  uint32_t depth = d.depth;
  for (uint32_t k = 0; k < d.depth; k++) {   // (the preopen: the Parent chain's end)
    const size_t s = root.rfind('/');
    if (s != std::string::npos && s > 0) root.resize(s);
  }
  bool allow_empty = false;
  int links = 0;
  size_t p = 0;
  for (;;) {
    if (p >= path.size() && !allow_empty) return ERRNO_NOENT;
    if (p < path.size() && path[p] == '/') {   // absolute: from the preopen
      allow_empty = true;
      cur = root;
      depth = 0;
      while (p < path.size() && path[p] == '/') p++;
    }
    if (d.kind != Fd::DIR) return ERRNO_NOTDIR;
    bool retry = false;
    while (!retry) {
      const size_t slash = path.find('/', p);
      const size_t pe = slash == std::string::npos ? path.size() : slash;
      const std::string part = path.substr(p, pe - p);
      size_t rem = pe;
      while (rem < path.size() && path[rem] == '/') rem++;
      const bool lastp = rem >= path.size() && slash == std::string::npos;
      if (!part.empty() && part[0] == '.') {
        if (part.size() == 1) {
          if (lastp) { *dir = cur; *last = "."; return ERRNO_SUCCESS; }
          p = rem;
          continue;
        }
        if (part == "..") {
          if (!depth) return ERRNO_NOTCAPABLE;
          cur.resize(cur.rfind('/'));
          depth--;
          p = rem;
          if (lastp) { *dir = cur; *last = "."; return ERRNO_SUCCESS; }
          continue;
        }
      }
      if (lastp && !(lookup & 1)) { *dir = cur; *last = part; return ERRNO_SUCCESS; }
      const std::string full = cur + "/" + part;
      struct stat st;
      if (::fstatat(AT_FDCWD, full.c_str(), &st, AT_SYMLINK_NOFOLLOW) != 0) {
        if (lastp) { *dir = cur; *last = part; return ERRNO_SUCCESS; }
        return from_errno(errno);
      }
      if (S_ISLNK(st.st_mode)) {   // the link's target, then the rest of the path
        if (++links >= kMaxNestedLinks) return ERRNO_LOOP;
        char tgt[4096];
        const ssize_t n = ::readlink(full.c_str(), tgt, sizeof tgt - 1);
        if (n < 0) return from_errno(errno);
        std::string np(tgt, size_t(n));
        if (rem < path.size()) {
          if (np.empty() || np.back() != '/') np += '/';
          np += path.substr(rem);
        }
        path = np;
        p = 0;
        retry = true;
        continue;
      }
      if (lastp) { *dir = cur; *last = part; return ERRNO_SUCCESS; }
      if (!S_ISDIR(st.st_mode)) return ERRNO_NOTDIR;
      cur = full;
      depth++;
      p = rem;
      if (p >= path.size()) { *dir = cur; *last = "."; return ERRNO_SUCCESS; }
    }
  }
}

inline uint32_t path_open(MemIO &m, const Env &cenv, Lane &lane, const uint64_t *a) {
  Env &env = const_cast<Env &>(cenv);   // (its blob cache)
  const int32_t dfd = int32_t(a[0]);
  const uint32_t dirflags = uint32_t(a[1]), pp = uint32_t(a[2]), plen = uint32_t(a[3]);
  const uint16_t of = uint16_t(a[4]), ff = uint16_t(a[7]);   // (the casts' raw widths)
  const uint64_t rb = a[5], ri = a[6];
  const uint32_t fdp = uint32_t(a[8]);
  if (!m.present()) return ERRNO_FAULT;
  if (dirflags & ~1u) return ERRNO_INVAL;
  if (of & ~15u) return ERRNO_INVAL;
  if ((rb & ~rights::ALL) || (ri & ~rights::ALL)) return ERRNO_INVAL;
  if (ff & ~31u) return ERRNO_INVAL;
  if (!in_bounds(m, pp, 1, plen)) return ERRNO_FAULT;
  if (!in_bounds(m, fdp, 4, 1)) return ERRNO_FAULT;
  Fd *d = fd_of(env, lane, dfd);
  if (!d) return ERRNO_BADF;
  uint64_t need = rights::PATH_OPEN;
  if (of & 1) need |= rights::PATH_CREATE_FILE;
  if (of & 8) need |= rights::PATH_FILESTAT_SET_SIZE;
  if (ff & 8) need |= rights::FD_SYNC;
  if (ff & 2) need |= rights::FD_DATASYNC;
  const bool rd = rb & (rights::FD_READ | rights::FD_READDIR);
  const bool wr = rb & (rights::FD_DATASYNC | rights::FD_WRITE | rights::FD_ALLOCATE |
                        rights::FD_FILESTAT_SET_SIZE);
  std::string path(plen, '\0'), dir, last;
  if (plen) m.read(pp, plen, reinterpret_cast<uint8_t *>(&path[0]));
  uint32_t e = resolve(*d, path, dirflags, &dir, &last);
  if (e) return e;
  if (!can(*d, need, rb | ri)) return ERRNO_NOTCAPABLE;
  const std::string full = last == "." ? dir : dir + "/" + last;
  struct stat st;
  const bool exists = ::fstatat(AT_FDCWD, full.c_str(), &st, AT_SYMLINK_NOFOLLOW) == 0;
  const int serr = errno;
  // openat(O_NOFOLLOW | ...) on a read-only mount: creating a file ROFS, O_EXCL of an
  // existing one EXIST, O_CREAT of a directory ISDIR, write access or O_TRUNC ROFS (O_CREAT
  // of an existing file just opens it)
  if (!exists) e = (of & 1) ? ERRNO_ROFS : from_errno(serr);
  else if ((of & 1) && (of & 4)) e = ERRNO_EXIST;
  else if (S_ISLNK(st.st_mode)) e = ERRNO_LOOP;
  else if ((of & 1) && S_ISDIR(st.st_mode)) e = ERRNO_ISDIR;   // (O_CREAT of a directory)
  else if ((of & 2) && !S_ISDIR(st.st_mode)) e = ERRNO_NOTDIR;
  else if (S_ISDIR(st.st_mode) && wr) e = ERRNO_ISDIR;
  else if (wr || (of & 8)) e = ERRNO_ROFS;
  std::shared_ptr<const Blob> blob;
  if (!e && S_ISREG(st.st_mode) && rd) {
    int err = 0;
    blob = env.blob(full, &err);
    if (!blob) e = from_errno(err);
  }
  if (e) return e;
  uint32_t nfd;   // Environ::generateRandomFdToNode
  do nfd = uint32_t(next_rand(lane)) & 0x7FFFFFFFu; while (lane.fds.count(nfd));
  Fd f;
  f.kind = S_ISDIR(st.st_mode) ? Fd::DIR : Fd::FILE;
  f.host = full;
  f.depth = d->depth + 1;
  f.rb = d->rb;   // VINode(FS, Node, Parent) takes its parent's rights
  f.ri = d->ri;
  f.blob = blob;
  lane.fds[nfd] = f;
  put_u32(m, fdp, nfd);
  return ERRNO_SUCCESS;
}

// iovec checks shared by fd_read and fd_write: the arrays, then each buffer (capped total)
inline uint32_t iovecs(MemIO &m, uint32_t iovs, uint32_t niov, uint32_t nptr,
                       std::vector<uint32_t> *bufs, std::vector<uint32_t> *lens) {
  if (!m.present()) return ERRNO_FAULT;
  if (niov > kIOVMax) return ERRNO_INVAL;
  if (!in_bounds(m, iovs, 8, niov)) return ERRNO_FAULT;
  if (!in_bounds(m, nptr, 4, 1)) return ERRNO_FAULT;
  bufs->resize(niov);
  lens->resize(niov);
  uint32_t total = 0;
  for (uint32_t k = 0; k < niov; k++) {
    const uint32_t b = get_u32(m, iovs + 8 * k), l = get_u32(m, iovs + 8 * k + 4);
    const uint32_t space = 0xFFFFFFFFu - total;      // capping total size
    const uint32_t len = l > space ? space : l;
    total += len;
    if (!in_bounds(m, b, 1, len)) return ERRNO_FAULT;
    (*bufs)[k] = b;
    (*lens)[k] = len;
  }
  return ERRNO_SUCCESS;
}

inline uint32_t fd_write(MemIO &m, const Env &env, Lane &lane, int32_t fd, uint32_t iovs, uint32_t niov,
                         uint32_t nwritten) {
  std::vector<uint32_t> bufs, lens;
  if (const uint32_t e = iovecs(m, iovs, niov, nwritten, &bufs, &lens)) return e;
  const Fd *f = fd_of(env, lane, fd);
  if (!f) return ERRNO_BADF;
  if (!can(*f, rights::FD_WRITE)) return ERRNO_NOTCAPABLE;
  if (f->kind != Fd::STDOUT && f->kind != Fd::STDERR) return ERRNO_BADF;
  std::string &out = lane.out[f->kind == Fd::STDOUT ? 0 : 1];
  uint32_t total = 0;
  for (uint32_t k = 0; k < niov; k++) {
    const size_t at = out.size();
    out.resize(at + lens[k]);
    if (lens[k]) m.read(bufs[k], lens[k], reinterpret_cast<uint8_t *>(&out[at]));
    total += lens[k];
  }
  put_u32(m, nwritten, total);
  return ERRNO_SUCCESS;
}

inline uint32_t fd_read(MemIO &m, const Env &env, Lane &lane, int32_t fd, uint32_t iovs, uint32_t niov,
                        uint32_t nread) {
  std::vector<uint32_t> bufs, lens;
  if (const uint32_t e = iovecs(m, iovs, niov, nread, &bufs, &lens)) return e;
  Fd *f = fd_of(env, lane, fd);
  if (!f) return ERRNO_BADF;
  if (!can(*f, rights::FD_READ)) return ERRNO_NOTCAPABLE;
  if (f->kind == Fd::DIR) return ERRNO_ISDIR;
  uint32_t got = 0;
  if (f->kind == Fd::FILE && f->blob) {   // (stdin: end of file)
    const std::vector<uint8_t> &b = f->blob->bytes;
    for (uint32_t k = 0; k < niov; k++) {
      const uint64_t left = f->off < b.size() ? b.size() - f->off : 0;
      const uint32_t n = uint32_t(std::min<uint64_t>(lens[k], left));
      if (n) m.write(bufs[k], n, b.data() + f->off);
      f->off += n;
      got += n;
      if (n < lens[k]) break;
    }
  }
  put_u32(m, nread, got);
  return ERRNO_SUCCESS;
}

inline uint32_t fd_seek(MemIO &m, const Env &env, Lane &lane, int32_t fd, int64_t off, uint32_t whence,
                        uint32_t p) {
  if (!m.present()) return ERRNO_FAULT;
  if (uint8_t(whence) > 2) return ERRNO_INVAL;   // cast<__wasi_whence_t> (u8)
  if (!in_bounds(m, p, 8, 1)) return ERRNO_FAULT;
  Fd *f = fd_of(env, lane, fd);
  if (!f) return ERRNO_BADF;
  if (!can(*f, rights::FD_SEEK)) return ERRNO_NOTCAPABLE;
  if (f->kind != Fd::FILE) return f->kind == Fd::DIR ? ERRNO_INVAL : ERRNO_SPIPE;
  const int64_t size = f->blob ? int64_t(f->blob->bytes.size()) : 0;
  const int64_t base = uint8_t(whence) == 0 ? 0 : uint8_t(whence) == 1 ? int64_t(f->off) : size;
  const int64_t n = int64_t(uint64_t(base) + uint64_t(off));
  if (n < 0 || (off > 0 && n < base)) return ERRNO_INVAL;   // lseek: EINVAL / overflow
  f->off = uint64_t(n);
  put_le(m, p, uint64_t(n), 8);
  return ERRNO_SUCCESS;
}

inline uint32_t fd_tell(MemIO &m, const Env &env, Lane &lane, int32_t fd, uint32_t p) {
  if (!m.present()) return ERRNO_FAULT;
  if (!in_bounds(m, p, 8, 1)) return ERRNO_FAULT;
  const Fd *f = fd_of(env, lane, fd);
  if (!f) return ERRNO_BADF;
  if (!can(*f, rights::FD_TELL)) return ERRNO_NOTCAPABLE;
  if (f->kind != Fd::FILE) return f->kind == Fd::DIR ? ERRNO_INVAL : ERRNO_SPIPE;
  put_le(m, p, f->off, 8);
  return ERRNO_SUCCESS;
}

inline uint32_t fd_close(const Env &env, Lane &lane, int32_t fd) {
  const Fd *f = fd_of(env, lane, fd);
  if (!f) return ERRNO_BADF;
  if (f->pre >= 0) return ERRNO_NOTSUP;
  lane.fds.erase(uint32_t(fd));
  return ERRNO_SUCCESS;
}

// __wasi_fdstat_t: u8 filetype @0, u16 flags @2, u64 rights_base @8, u64 inheriting @16
inline uint32_t fd_fdstat_get(MemIO &m, const Env &env, Lane &lane, int32_t fd, uint32_t p) {
  if (!m.present()) return ERRNO_FAULT;
  if (!in_bounds(m, p, 24, 1)) return ERRNO_FAULT;
  const Fd *f = fd_of(env, lane, fd);
  if (!f) return ERRNO_BADF;
  put_le(m, p + 8, f->rb, 8);
  put_le(m, p + 16, f->ri, 8);
  uint8_t ft = FILETYPE_CHARACTER_DEVICE;
  if (f->kind == Fd::DIR || f->kind == Fd::FILE) {
    struct stat st;
    if (const int e = stat_of(*f, &st)) return from_errno(e);
    ft = filetype_of(st.st_mode);
  }
  put_le(m, p, ft, 1);
  put_le(m, p + 2, 0, 2);   // (O_RDONLY opens and the captures carry no fdflags)
  return ERRNO_SUCCESS;
}

inline uint32_t fd_fdstat_set_flags(const Env &env, Lane &lane, int32_t fd, uint32_t flags) {
  if (uint16_t(flags) & ~31u) return ERRNO_INVAL;
  const Fd *f = fd_of(env, lane, fd);
  if (!f) return ERRNO_BADF;
  uint64_t need = rights::FD_FDSTAT_SET_FLAGS;
  if (flags & 2) need |= rights::FD_DATASYNC;
  if (flags & (8 | 16)) need |= rights::FD_SYNC;
  if (!can(*f, need)) return ERRNO_NOTCAPABLE;
  return ERRNO_SUCCESS;
}

// __wasi_filestat_t: dev @0, ino @8, u8 filetype @16, nlink @24, size @32, atim @40,
// mtim @48, ctim @56
inline void put_filestat(MemIO &m, uint32_t p, const struct stat &st) {
  put_le(m, p, uint64_t(st.st_dev), 8);
  put_le(m, p + 8, uint64_t(st.st_ino), 8);
  put_le(m, p + 16, filetype_of(st.st_mode), 1);
  put_le(m, p + 24, uint64_t(st.st_nlink), 8);
  put_le(m, p + 32, uint64_t(st.st_size), 8);
  put_le(m, p + 40, ns_of(st.st_atim), 8);
  put_le(m, p + 48, ns_of(st.st_mtim), 8);
  put_le(m, p + 56, ns_of(st.st_ctim), 8);
}

inline uint32_t fd_filestat_get(MemIO &m, const Env &env, Lane &lane, int32_t fd, uint32_t p) {
  if (!m.present()) return ERRNO_FAULT;
  if (!in_bounds(m, p, 64, 1)) return ERRNO_FAULT;
  const Fd *f = fd_of(env, lane, fd);
  if (!f) return ERRNO_BADF;
  if (!can(*f, rights::FD_FILESTAT_GET)) return ERRNO_NOTCAPABLE;
  struct stat st;
  memset(&st, 0, sizeof st);
  if (f->kind == Fd::DIR || f->kind == Fd::FILE) {
    if (const int e = stat_of(*f, &st)) return from_errno(e);
  } else {   // the capture: a character device with no times
    st.st_mode = S_IFCHR;
    st.st_nlink = 1;
  }
  put_filestat(m, p, st);
  return ERRNO_SUCCESS;
}

inline uint32_t path_filestat_get(MemIO &m, const Env &env, Lane &lane, const uint64_t *a) {
  const int32_t fd = int32_t(a[0]);
  const uint32_t flags = uint32_t(a[1]), pp = uint32_t(a[2]), plen = uint32_t(a[3]), p = uint32_t(a[4]);
  if (!m.present()) return ERRNO_FAULT;
  if (flags & ~1u) return ERRNO_INVAL;
  if (!in_bounds(m, pp, 1, plen)) return ERRNO_FAULT;
  if (!in_bounds(m, p, 64, 1)) return ERRNO_FAULT;
  const Fd *d = fd_of(env, lane, fd);
  if (!d) return ERRNO_BADF;
  std::string path(plen, '\0'), dir, last;
  if (plen) m.read(pp, plen, reinterpret_cast<uint8_t *>(&path[0]));
  if (const uint32_t e = resolve(*d, path, flags, &dir, &last)) return e;
  if (!can(*d, rights::PATH_FILESTAT_GET)) return ERRNO_NOTCAPABLE;
  const std::string full = last == "." ? dir : dir + "/" + last;
  struct stat st;
  if (::fstatat(AT_FDCWD, full.c_str(), &st, (flags & 1) ? 0 : AT_SYMLINK_NOFOLLOW) != 0)
    return from_errno(errno);
  put_filestat(m, p, st);
  return ERRNO_SUCCESS;
}

inline uint32_t clock_get(MemIO &m, const Env &env, Lane &lane, uint32_t id, uint32_t p, bool res) {
  static const clockid_t ids[4] = {CLOCK_REALTIME, CLOCK_MONOTONIC, CLOCK_PROCESS_CPUTIME_ID,
                                   CLOCK_THREAD_CPUTIME_ID};
  if (!m.present()) return ERRNO_FAULT;
  if (!in_bounds(m, p, 8, 1)) return ERRNO_FAULT;
  if (id > 3) return ERRNO_INVAL;   // cast<__wasi_clockid_t>
  struct timespec t = {0, 1};
  uint64_t v;
  if (env.fixed_clock) {
    v = res ? 1 : env.clock_ns + 1000ull * lane.clock_calls++;
  } else {
    if (res) ::clock_getres(ids[id], &t);
    else ::clock_gettime(ids[id], &t);
    v = ns_of(t);
  }
  put_le(m, p, v, 8);
  return ERRNO_SUCCESS;
}

inline uint32_t random_get(MemIO &m, const Env &env, Lane &lane, uint32_t p, uint32_t len) {
  if (!m.present()) return ERRNO_FAULT;
  if (!in_bounds(m, p, 1, len)) return ERRNO_FAULT;
  fs_ready(env, lane);
  for (uint32_t k = 0; k < len; k += 4) {   // 32-bit draws, the last cut to what is left
    const uint32_t v = uint32_t(next_rand(lane));
    put_le(m, p + k, v, std::min<uint32_t>(4, len - k));
  }
  return ERRNO_SUCCESS;
}

// fd_prestat_get: __wasi_prestat_t {u8 tag; u32 pr_name_len} (the 3 padding bytes untouched)
inline uint32_t fd_prestat_get(MemIO &m, const Env &env, Lane &lane, int32_t fd, uint32_t ptr) {
  if (!m.present()) return ERRNO_FAULT;
  if (!in_bounds(m, ptr, 8, 1)) return ERRNO_FAULT;
  const Fd *f = fd_of(env, lane, fd);
  if (!f) return ERRNO_BADF;
  if (f->pre < 0) return ERRNO_INVAL;                   // a node with no name
  put_le(m, ptr, kPreopenTypeDir, 1);
  put_u32(m, ptr + 4, uint32_t(env.preopens[size_t(f->pre)].size()));
  return ERRNO_SUCCESS;
}

inline uint32_t fd_prestat_dir_name(MemIO &m, const Env &env, Lane &lane, int32_t fd, uint32_t buf, uint32_t len) {
  if (!m.present()) return ERRNO_FAULT;
  if (!in_bounds(m, buf, 1, len)) return ERRNO_FAULT;
  const Fd *f = fd_of(env, lane, fd);
  if (!f) return ERRNO_BADF;
  if (f->pre < 0) return ERRNO_INVAL;
  const std::string &name = env.preopens[size_t(f->pre)];
  const uint32_t k = uint32_t(name.size()) < len ? uint32_t(name.size()) : len;
  if (k) m.write(buf, k, reinterpret_cast<const uint8_t *>(name.data()));
  return ERRNO_SUCCESS;
}

// Run WASI function `f` for one instance. a: the operands (i32 zero-extended, i64 whole);
// *ret: the errno result. Returns 0, or the ErrCode that ends the instance (Terminated for
// proc_exit).
inline uint8_t call(int f, const Env &env, Lane &lane, MemIO &m, const uint64_t *a, uint32_t *ret) {
  const uint32_t a0 = uint32_t(a[0]), a1 = uint32_t(a[1]), a2 = uint32_t(a[2]), a3 = uint32_t(a[3]);
  switch (f) {
  case ARGS_GET: *ret = list_get(m, lane.own_args ? lane.args : env.args, a0, a1); return 0;
  case ARGS_SIZES_GET: *ret = list_sizes(m, lane.own_args ? lane.args : env.args, a0, a1); return 0;
  case ENVIRON_GET: *ret = list_get(m, env.envs, a0, a1); return 0;
  case ENVIRON_SIZES_GET: *ret = list_sizes(m, env.envs, a0, a1); return 0;
  case FD_WRITE: *ret = fd_write(m, env, lane, int32_t(a0), a1, a2, a3); return 0;
  case PROC_EXIT: lane.exit_code = a0; return kTerminated;
  case SCHED_YIELD: *ret = ERRNO_SUCCESS; return 0;
  case FD_PRESTAT_GET: *ret = fd_prestat_get(m, env, lane, int32_t(a0), a1); return 0;
  case FD_PRESTAT_DIR_NAME: *ret = fd_prestat_dir_name(m, env, lane, int32_t(a0), a1, a2); return 0;
  case PATH_OPEN: *ret = path_open(m, env, lane, a); return 0;
  case FD_READ: *ret = fd_read(m, env, lane, int32_t(a0), a1, a2, a3); return 0;
  case FD_SEEK: *ret = fd_seek(m, env, lane, int32_t(a0), int64_t(a[1]), a2, a3); return 0;
  case FD_TELL: *ret = fd_tell(m, env, lane, int32_t(a0), a1); return 0;
  case FD_CLOSE: *ret = fd_close(env, lane, int32_t(a0)); return 0;
  case FD_FDSTAT_GET: *ret = fd_fdstat_get(m, env, lane, int32_t(a0), a1); return 0;
  case FD_FDSTAT_SET_FLAGS: *ret = fd_fdstat_set_flags(env, lane, int32_t(a0), a1); return 0;
  case FD_FILESTAT_GET: *ret = fd_filestat_get(m, env, lane, int32_t(a0), a1); return 0;
  case PATH_FILESTAT_GET: *ret = path_filestat_get(m, env, lane, a); return 0;
  case CLOCK_TIME_GET: *ret = clock_get(m, env, lane, a0, a2, false); return 0;
  case CLOCK_RES_GET: *ret = clock_get(m, env, lane, a0, a1, true); return 0;
  case RANDOM_GET: *ret = random_get(m, env, lane, a0, a1); return 0;
  }
  return 0x8D;   // HostFuncFailed
}

// the operands of a call from its cells (i32: one cell, i64: two, little end first)
inline void args_of_cells(const std::vector<uint8_t> &params, const uint32_t *cells, uint64_t *a) {
  uint32_t c = 0;
  for (size_t k = 0; k < params.size() && k < kMaxArgs; k++) {
    if (params[k] == 0x7E) {
      a[k] = uint64_t(cells[c]) | uint64_t(cells[c + 1]) << 32;
      c += 2;
    } else {
      a[k] = cells[c++];
    }
  }
}

}  // namespace wbw
