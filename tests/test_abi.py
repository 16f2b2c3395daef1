"""The drop-in boundary: libwasmedge_batch.so loads on a GPU-less host and exports every
entry point include/wasmedge_batch.h declares (no compute calls -- those are -m gpu)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "wasmedge_batch.h")
LIB = os.path.join(ROOT, "wasmedge_amd", "libwasmedge_batch.so")


def declared():
    """Entry points the library must export (header-inline helpers excluded)."""
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    inline = set(re.findall(r"static inline [^(]*\b(WasmEdge_Batch[A-Za-z]+)\s*\(", src))
    return sorted(set(re.findall(r"\b(WasmEdge_Batch[A-Za-z]+)\s*\(", src)) - inline)


def test_header_declares_api():
    names = declared()
    for must in ["WasmEdge_BatchCreate", "WasmEdge_BatchExecute", "WasmEdge_BatchSetArgs",
                 "WasmEdge_BatchReset", "WasmEdge_BatchRun", "WasmEdge_BatchResults",
                 "WasmEdge_BatchMemoryHash", "WasmEdge_BatchGetMemory",
                 "WasmEdge_BatchDelete", "WasmEdge_BatchGetLastError"]:
        assert must in names


def test_library_exports_every_declared_symbol(built):
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert missing == []
    dyn = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True,
                         text=True, check=True).stdout
    exported = set(l.split()[-1] for l in dyn.splitlines() if l.strip())
    assert set(declared()) <= exported
    # nothing but the C ABI leaks out of the library's public surface
    leaked = [s for s in exported if s.startswith("_Z") and "wb_" in s]
    assert leaked == []


def _tree_hash():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "wasmedge_amd", "csrc"))
    import srchash
    return srchash.source_hash()


def test_library_matches_the_sources(built):
    """The built library carries the hash of the sources it came from (csrc/srchash.py),
    and it is the checked-out tree's: the file, and the library a process loads."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "wasmedge_amd", "csrc"))
    import srchash
    assert srchash.embedded_hash(LIB) == _tree_hash()
    from wasmedge_amd import batch
    batch.lib().WasmEdge_BatchGetBuildHash.restype = ctypes.c_char_p
    assert batch.lib().WasmEdge_BatchGetBuildHash().decode() == _tree_hash()


@pytest.mark.gpu
def test_gpu_loaded_library_is_head(built):
    """On the GPU box: the library this process loaded (and runs every GPU test through)
    was built from these sources -- no stale shipped build."""
    from wasmedge_amd import batch
    L = batch.lib()
    L.WasmEdge_BatchGetBuildHash.restype = ctypes.c_char_p
    assert L.WasmEdge_BatchGetBuildHash().decode() == _tree_hash()
    ctx = batch.BatchContext(open(os.path.join(ROOT, "tests", "golden", "fibonacci.wasm"), "rb").read(),
                             64, device=0)
    try:
        rets, st, cnt = ctx.execute("fib", batch.make_values([[10]] * 64, [batch.I32]), 1)
        assert (st == 0).all()
    finally:
        ctx.close()


DRIVER = os.path.join(ROOT, "tests", "c", "abi_driver")


def test_c_driver_is_built(built):
    """tests/c/abi_driver.c -- a plain C embedder of the ABI -- is built against the header
    and links the library (run on the GPU below)."""
    assert os.access(DRIVER, os.X_OK)
    out = subprocess.run(["ldd", DRIVER], capture_output=True, text=True).stdout
    assert "libwasmedge_batch.so" in out and "not found" not in out


@pytest.mark.gpu
def test_gpu_c_driver(built):
    """A C program calls the ABI on the GPU (no ctypes): Create / Execute / the staged
    SetArgs-Reset-Run-Results path / MemoryHash / FuncNotFound, on one device and on two
    shards, every result and instruction count checked in C against fib and the reference's
    counting rule."""
    r = subprocess.run([DRIVER, os.path.join(ROOT, "tests", "golden", "fibonacci.wasm")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "one device: 1000 instances ok" in r.stdout and "two shards: 1000 instances ok" in r.stdout


def test_null_context_is_wrong_workflow(built):
    """Reference C API: NULL context -> WrongVMWorkflow (lib/api/wasmedge.cpp:266-277).
    Exercised without a GPU: no device call happens before the NULL check."""
    from wasmedge_amd import batch
    L = batch.lib()
    assert L.WasmEdge_BatchRun(None, None).Code == 0x04
    assert L.WasmEdge_BatchReset(None, None).Code == 0x04
    assert L.WasmEdge_BatchGetInstanceCount(None) == 0


def test_create_rejects_malformed_module(built):
    """Load/validate failures come back as the reference ErrCode, before any device
    allocation (lib/loader, ErrCode::MalformedMagic = 0x21 etc.)."""
    from wasmedge_amd import batch
    import pytest
    with pytest.raises(batch.WasmEdgeError) as e:
        batch.BatchContext(b"\x00asn\x01\x00\x00\x00", 64)
    assert e.value.code == 0x23          # ErrCode::MalformedMagic (enum.inc:603)


def test_ctypes_layouts_match_the_header(tmp_path):
    """The Python mirror's structures have the C header's layout (gcc on the header):
    a mismatch would hand the library garbage pointers."""
    import ctypes
    import subprocess
    from wasmedge_amd import batch as b
    src = tmp_path / "layout.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "%s/include/wasmedge_batch.h"\n'
                   'int main(void) {\n'
                   '  printf("%%zu %%zu %%zu %%zu %%zu %%zu %%zu\\n", sizeof(WasmEdge_BatchConfigure),\n'
                   '         offsetof(WasmEdge_BatchConfigure, CostTable), offsetof(WasmEdge_BatchConfigure, MemoryGranule),\n'
                   '         offsetof(WasmEdge_BatchConfigure, HostThreads), offsetof(WasmEdge_BatchConfigure, MemoryPoolBytes),\n'
                   '         offsetof(WasmEdge_BatchConfigure, Devices), offsetof(WasmEdge_BatchConfigure, Partition));\n'
                   '  printf("%%zu %%zu %%zu\\n", sizeof(WasmEdge_BatchImport), offsetof(WasmEdge_BatchImport, Value),\n'
                   '         offsetof(WasmEdge_BatchImport, Mutable));\n'
                   '  printf("%%zu\\n", sizeof(WasmEdge_Value));\n'
                   '  return 0;\n}\n' % ROOT)
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-o", str(exe), str(src)])
    got = [list(map(int, line.split())) for line in subprocess.check_output([str(exe)]).decode().splitlines()]
    C, I = b._Conf, b._Import
    assert got[0] == [ctypes.sizeof(C), C.CostTable.offset, C.MemoryGranule.offset, C.HostThreads.offset,
                      C.MemoryPoolBytes.offset, C.Devices.offset, C.Partition.offset]
    assert got[1] == [ctypes.sizeof(I), I.Value.offset, I.Mutable.offset]
    assert got[2] == [ctypes.sizeof(b._Value)]


REF_API = "/root/reference/include"


@pytest.mark.skipif(not os.path.isdir(REF_API), reason="reference tree absent (GPU box)")
def test_integration_snippets_compile_after_the_reference_header(tmp_path):
    """INTEGRATION.md's C snippets, with the reference's own C API header included first:
    its WasmEdge_Value / String / Result then serve both APIs (the WASMEDGE_C_API_H guard
    in include/wasmedge_batch.h). The header is used as installed: include/api/wasmedge/
    wasmedge.h next to the C enum headers of include/common/ it includes, and version.h made
    from version.h.in the way the reference's configure_file makes it. Compile only -- no
    reference code is built or run."""
    inc = tmp_path / "inc" / "wasmedge"
    inc.mkdir(parents=True)
    for f in ("enum_configure.h", "enum_errcode.h", "enum_types.h", "enum.inc"):
        (inc / f).symlink_to(os.path.join(REF_API, "common", f))
    for f in ("wasmedge.h", "int128.h"):
        (inc / f).symlink_to(os.path.join(REF_API, "api", "wasmedge", f))
    ver = open(os.path.join(REF_API, "api", "wasmedge", "version.h.in")).read()
    for k, v in {"${CPACK_PACKAGE_VERSION}": "0.9.1", "${WASMEDGE_VERSION_MAJOR}": "0",
                 "${WASMEDGE_VERSION_MINOR}": "9", "${WASMEDGE_VERSION_PATCH}": "1"}.items():
        ver = ver.replace(k, v)
    (inc / "version.h").write_text(ver)
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```c\n(.*?)```", doc, re.S)
    assert len(blocks) >= 2
    body, funcs = [], []
    for b in blocks:
        lines = [ln for ln in b.splitlines() if not ln.startswith("#include")]
        text = "\n".join(lines)
        # host-function definitions stay at file scope, statements go into a function
        if "WasmEdge_Result MemSum(" in text:
            head, _, rest = text.partition("WasmEdge_String mod")
            funcs.append(head)
            body.append("WasmEdge_String mod" + rest)
        else:
            body.append(text)
    src = ("#include <stdio.h>\n#include <stdlib.h>\n#include <wasmedge/wasmedge.h>\n"
           '#include "wasmedge_batch.h"\n' + "\n".join(funcs) +
           "\nint use(const uint8_t *wasm_bytes, uint32_t wasm_len) {\n" + "\n".join(body) +
           "\nreturn 0;\n}\n")
    c = tmp_path / "snippet.c"
    c.write_text(src)
    r = subprocess.run(["gcc", "-std=gnu11", "-Wall", "-Werror", "-Wno-unused-variable", "-c",
                        "-I", str(tmp_path / "inc"), "-I", os.path.join(ROOT, "include"),
                        str(c), "-o", str(tmp_path / "snippet.o")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_gpu_boundary_errors(built):
    """Call-level errors of WasmEdge_BatchExecute / SetArgs, as the reference VM reports
    them (executor.cpp:88-100, vm.cpp): FuncNotFound (0x05) for an unknown export,
    FuncSigMismatch (0x83) for a wrong parameter count or type, WrongVMWorkflow (0x04) for
    Results before a Run; per-instance traps never surface here."""
    import numpy as np
    from wasmedge_amd import batch
    with open(os.path.join(ROOT, "tests", "golden", "fibonacci.wasm"), "rb") as f:
        fib = f.read()
    ctx = batch.BatchContext(fib, 64, device=0)
    try:
        with pytest.raises(batch.WasmEdgeError) as e:
            ctx.results(1)
        assert e.value.code == 0x04
        with pytest.raises(batch.WasmEdgeError) as e:
            ctx.execute("nope", batch.make_values([[1]] * 64, [batch.I32]), 1)
        assert e.value.code == 0x05
        with pytest.raises(batch.WasmEdgeError) as e:
            ctx.execute("fib", batch.make_values([[1, 2]] * 64, [batch.I32, batch.I32]), 1)
        assert e.value.code == 0x83
        with pytest.raises(batch.WasmEdgeError) as e:
            ctx.execute("fib", batch.make_values([[1]] * 64, [batch.I64]), 1)
        assert e.value.code == 0x83
        rets, st, cnt = ctx.execute("fib", batch.make_values([[10]] * 64, [batch.I32]), 1)
        # fibonacci.wasm counts fib(0) = fib(1) = 1 (fib 8 -> 34, the examples README)
        assert (st == 0).all() and list(set(batch.ret_ints(rets)[:, 0])) == [89]
        assert np.all(cnt == cnt[0])
    finally:
        ctx.close()
