"""Hash of the sources libwasmedge_batch.so is built from (csrc/ and the C ABI header).

The Makefile embeds it into the library (build/srchash.h -> WasmEdge_BatchGetBuildHash),
__graft_entry__.build() rebuilds when the library's embedded hash differs from the tree's
(so a shipped library never runs stale against its sources), and a GPU test asserts that
the library a process loaded is the one built from the checked-out sources.

    python3 srchash.py            print the hash
    python3 srchash.py OUT.h      write the header the library includes
"""
import glob
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PATTERNS = ("*.cpp", "*.h", "*.hip", "*.inc", "*.py", "Makefile")
MARK = b"WB_SRC_HASH="


def source_files():
    files = set()
    for p in PATTERNS:
        files.update(glob.glob(os.path.join(HERE, p)))
    files.add(os.path.join(ROOT, "include", "wasmedge_batch.h"))
    return sorted(os.path.relpath(f, ROOT) for f in files)


def source_hash():
    h = hashlib.sha256()
    for rel in source_files():
        with open(os.path.join(ROOT, rel), "rb") as f:
            data = f.read()
        h.update(rel.replace(os.sep, "/").encode() + b"\0" + data + b"\0")
    return h.hexdigest()[:32]


def embedded_hash(lib_path):
    """The hash a built library carries (read from the file, no dlopen), or None."""
    try:
        with open(lib_path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(MARK)
    return data[i + len(MARK):i + len(MARK) + 32].decode() if i >= 0 else None


if __name__ == "__main__":
    if len(sys.argv) > 1:
        text = '#define WB_SRC_HASH "%s"\n' % source_hash()
        old = open(sys.argv[1]).read() if os.path.exists(sys.argv[1]) else ""
        if old != text:   # (an unchanged hash does not touch the file: no needless rebuild)
            with open(sys.argv[1], "w") as f:
                f.write(text)
    else:
        print(source_hash())
