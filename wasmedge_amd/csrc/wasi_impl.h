// wasi_impl.h -- the built-in WASI subset (wasi_snapshot_preview1) served on the host
// for lanes that yield at a WASI import. One restatement, two users: the product
// library (wasi.cpp, memory through the host-call round's wave view) and the test
// emulator (emu.cpp, contiguous memory). Semantics follow the reference's host functions
// (lib/host/wasi/wasifunc.cpp) over its Environ (include/host/wasi/environ.h) with the
// default stdio rights (lib/host/wasi/environ.cpp:38-46):
//   args_get / args_sizes_get      wasifunc.cpp:314-372, environ.h:85-114
//   environ_get / environ_sizes_get wasifunc.cpp:374-433, environ.h:127-157
//   fd_write                       wasifunc.cpp:990-1046; fd 1/2 are captured per
//                                  instance, fd 0 is NOTCAPABLE (stdin has no write right,
//                                  vinode.h:337-343), other fds BADF (no preopens here)
//   proc_exit                      wasifunc.cpp:1550-1554 (exit code, then Terminated)
//   sched_yield                    wasifunc.cpp:1571-1576
//   fd_prestat_get                 wasifunc.cpp:746-766, environ.h:385-399: BADF for an fd
//                                  with no node, INVAL for the stdio nodes (no name), else
//                                  tag DIR + the preopen's name length
//   fd_prestat_dir_name            wasifunc.cpp:724-744, environ.h:406-420: the name's
//                                  first min(name, len) bytes
// Args may be given per instance (WasmEdge_BatchWASISetInstanceArgs); the reference builds
// one Environ per VM, so per-instance args are per-VM args.
// Every pointer is bounds-checked like MemoryInstance::getPointer (memory.h:226-233:
// Offset + sizeof(T) * Count <= size, the product in 32 bits) before anything is written.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace wbw {

enum : uint32_t {                       // thirdparty/wasi/api.hpp
  ERRNO_SUCCESS = 0, ERRNO_BADF = 8, ERRNO_FAULT = 21, ERRNO_INVAL = 28, ERRNO_NOTCAPABLE = 76
};
constexpr uint8_t kPreopenTypeDir = 0;  // __WASI_PREOPENTYPE_DIR
constexpr uint32_t kIOVMax = 1024;      // include/host/wasi/environ.h:33
constexpr uint32_t kMaxArgs = 4;        // operands of the widest function in the subset
constexpr uint8_t kTerminated = 0x01;   // ErrCode::Terminated (enum.inc)

enum Fn { ARGS_GET, ARGS_SIZES_GET, ENVIRON_GET, ENVIRON_SIZES_GET, FD_WRITE, PROC_EXIT,
          SCHED_YIELD, FD_PRESTAT_GET, FD_PRESTAT_DIR_NAME, NUM_FNS };

// configuration shared by every instance (WasmEdge_ImportObjectCreateWASI's Args/Envs/
// Preopens): preopens are the guest names of fds 3, 4, ... (environ.cpp:54-93)
struct Env {
  std::vector<std::string> args, envs, preopens;
};
// per-instance WASI state: captured stdout/stderr, the proc_exit code and, when the
// instance has args of its own, those args
struct Lane {
  std::string out[2];
  uint32_t exit_code = 0;
  bool own_args = false;
  std::vector<std::string> args;
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

// one instance's linear memory
struct MemIO {
  virtual ~MemIO() {}
  virtual bool present() = 0;                     // the module has a memory
  virtual uint64_t size() = 0;                    // bytes (pages * 64 KiB)
  virtual bool read(uint32_t off, uint32_t len, uint8_t *dst) = 0;    // in bounds only
  virtual bool write(uint32_t off, uint32_t len, const uint8_t *src) = 0;
};

// The import `name` of module wasi_snapshot_preview1 with value types (0x7F = i32) `params`
// -> `results`, or -1 if not in the subset / of another signature (then the import stays
// unbound and a lane reaching it reports 0xB1).
inline int lookup(const std::string &name, const std::vector<uint8_t> &params,
                  const std::vector<uint8_t> &results) {
  struct S { const char *n; Fn f; uint8_t np, nr; };
  static const S tab[] = {{"args_get", ARGS_GET, 2, 1},
                          {"args_sizes_get", ARGS_SIZES_GET, 2, 1},
                          {"environ_get", ENVIRON_GET, 2, 1},
                          {"environ_sizes_get", ENVIRON_SIZES_GET, 2, 1},
                          {"fd_write", FD_WRITE, 4, 1},
                          {"proc_exit", PROC_EXIT, 1, 0},
                          {"sched_yield", SCHED_YIELD, 0, 1},
                          {"fd_prestat_get", FD_PRESTAT_GET, 2, 1},
                          {"fd_prestat_dir_name", FD_PRESTAT_DIR_NAME, 3, 1}};
  for (const S &s : tab) {
    if (name != s.n) continue;
    if (params.size() != s.np || results.size() != s.nr) return -1;
    for (uint8_t t : params) if (t != 0x7F) return -1;
    for (uint8_t t : results) if (t != 0x7F) return -1;
    return s.f;
  }
  return -1;
}

inline bool in_bounds(MemIO &m, uint32_t off, uint32_t size, uint32_t count) {
  const uint32_t bytes = size * count;   // getPointer: uint32 ByteSize
  return uint64_t(off) + bytes <= m.size();
}
inline void put_u32(MemIO &m, uint32_t off, uint32_t v) {
  const uint8_t b[4] = {uint8_t(v), uint8_t(v >> 8), uint8_t(v >> 16), uint8_t(v >> 24)};
  m.write(off, 4, b);
}
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

inline uint32_t fd_write(MemIO &m, Lane &lane, int32_t fd, uint32_t iovs, uint32_t niov,
                         uint32_t nwritten) {
  if (!m.present()) return ERRNO_FAULT;
  if (niov > kIOVMax) return ERRNO_INVAL;
  if (!in_bounds(m, iovs, 8, niov)) return ERRNO_FAULT;
  if (!in_bounds(m, nwritten, 4, 1)) return ERRNO_FAULT;
  std::vector<uint32_t> bufs(niov), lens(niov);
  uint32_t total = 0;
  for (uint32_t k = 0; k < niov; k++) {
    const uint32_t b = get_u32(m, iovs + 8 * k), l = get_u32(m, iovs + 8 * k + 4);
    const uint32_t space = 0xFFFFFFFFu - total;      // capping total size
    const uint32_t len = l > space ? space : l;
    total += len;
    if (!in_bounds(m, b, 1, len)) return ERRNO_FAULT;
    bufs[k] = b;
    lens[k] = len;
  }
  if (fd == 0) return ERRNO_NOTCAPABLE;
  if (fd != 1 && fd != 2) return ERRNO_BADF;
  std::string &out = lane.out[fd - 1];
  for (uint32_t k = 0; k < niov; k++) {
    const size_t at = out.size();
    out.resize(at + lens[k]);
    if (lens[k]) m.read(bufs[k], lens[k], reinterpret_cast<uint8_t *>(&out[at]));
  }
  put_u32(m, nwritten, total);
  return ERRNO_SUCCESS;
}

// the node behind fd: -1 none, 0..2 stdio, 3.. preopen k - 3 (Environ::getNodeOrNull)
inline int node_of(const Env &env, int32_t fd) {
  if (fd < 0) return -1;
  if (fd <= 2) return fd;
  return uint64_t(fd) - 3 < env.preopens.size() ? fd : -1;
}

// __wasi_prestat_t {u8 tag; u32 pr_name_len} (8 bytes; the 3 padding bytes untouched)
inline uint32_t fd_prestat_get(MemIO &m, const Env &env, int32_t fd, uint32_t ptr) {
  if (!m.present()) return ERRNO_FAULT;
  if (!in_bounds(m, ptr, 8, 1)) return ERRNO_FAULT;
  const int n = node_of(env, fd);
  if (n < 0) return ERRNO_BADF;
  if (n <= 2) return ERRNO_INVAL;                       // stdio nodes have no name
  const std::string &name = env.preopens[n - 3];
  const uint8_t tag = kPreopenTypeDir;
  m.write(ptr, 1, &tag);
  put_u32(m, ptr + 4, uint32_t(name.size()));
  return ERRNO_SUCCESS;
}

inline uint32_t fd_prestat_dir_name(MemIO &m, const Env &env, int32_t fd, uint32_t buf, uint32_t len) {
  if (!m.present()) return ERRNO_FAULT;
  if (!in_bounds(m, buf, 1, len)) return ERRNO_FAULT;
  const int n = node_of(env, fd);
  if (n < 0) return ERRNO_BADF;
  if (n <= 2) return ERRNO_INVAL;
  const std::string &name = env.preopens[n - 3];
  const uint32_t k = uint32_t(name.size()) < len ? uint32_t(name.size()) : len;
  if (k) m.write(buf, k, reinterpret_cast<const uint8_t *>(name.data()));
  return ERRNO_SUCCESS;
}

// Run WASI function `f` for one instance. args: i32 operands; *ret: the errno result.
// Returns 0, or the ErrCode that ends the instance (Terminated for proc_exit).
inline uint8_t call(int f, const Env &env, Lane &lane, MemIO &m, const uint32_t *a, uint32_t *ret) {
  switch (f) {
  case ARGS_GET: *ret = list_get(m, lane.own_args ? lane.args : env.args, a[0], a[1]); return 0;
  case ARGS_SIZES_GET: *ret = list_sizes(m, lane.own_args ? lane.args : env.args, a[0], a[1]); return 0;
  case ENVIRON_GET: *ret = list_get(m, env.envs, a[0], a[1]); return 0;
  case ENVIRON_SIZES_GET: *ret = list_sizes(m, env.envs, a[0], a[1]); return 0;
  case FD_WRITE: *ret = fd_write(m, lane, int32_t(a[0]), a[1], a[2], a[3]); return 0;
  case PROC_EXIT: lane.exit_code = a[0]; return kTerminated;
  case SCHED_YIELD: *ret = ERRNO_SUCCESS; return 0;
  case FD_PRESTAT_GET: *ret = fd_prestat_get(m, env, int32_t(a[0]), a[1]); return 0;
  case FD_PRESTAT_DIR_NAME: *ret = fd_prestat_dir_name(m, env, int32_t(a[0]), a[1], a[2]); return 0;
  }
  return 0x8D;   // HostFuncFailed
}

}  // namespace wbw
