"""The drop-in boundary: libwasmedge_batch.so loads on a GPU-less host and exports every
entry point include/wasmedge_batch.h declares (no compute calls -- those are -m gpu)."""
import ctypes
import os
import re
import subprocess

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "wasmedge_batch.h")
LIB = os.path.join(ROOT, "wasmedge_amd", "libwasmedge_batch.so")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(WasmEdge_Batch[A-Za-z]+)\s*\(", src)))


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
                   '  printf("%%zu %%zu %%zu %%zu\\n", sizeof(WasmEdge_BatchConfigure),\n'
                   '         offsetof(WasmEdge_BatchConfigure, CostTable), offsetof(WasmEdge_BatchConfigure, MemoryGranule),\n'
                   '         offsetof(WasmEdge_BatchConfigure, HostThreads));\n'
                   '  printf("%%zu %%zu %%zu\\n", sizeof(WasmEdge_BatchImport), offsetof(WasmEdge_BatchImport, Value),\n'
                   '         offsetof(WasmEdge_BatchImport, Mutable));\n'
                   '  printf("%%zu\\n", sizeof(WasmEdge_Value));\n'
                   '  return 0;\n}\n' % ROOT)
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-o", str(exe), str(src)])
    got = [list(map(int, line.split())) for line in subprocess.check_output([str(exe)]).decode().splitlines()]
    C, I = b._Conf, b._Import
    assert got[0] == [ctypes.sizeof(C), C.CostTable.offset, C.MemoryGranule.offset, C.HostThreads.offset]
    assert got[1] == [ctypes.sizeof(I), I.Value.offset, I.Mutable.offset]
    assert got[2] == [ctypes.sizeof(b._Value)]
