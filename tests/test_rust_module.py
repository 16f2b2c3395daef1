"""A compiled Rust/WASI module from the reference (tools/wasmedge/examples/add.wasm,
fixture tests/golden/rust_add.wasm, 1.7 MB): the loader, validator and lowering over a
real toolchain's output (hundreds of functions, WASI imports that `add` never reaches on
non-overflowing operands). Known answer: `wasmedge --reactor add.wasm add 2 2` -> 4
(docs/book/en/src/extend/build_for_android.md:70-71). Per-lane operands are checked
against the oracle: status, result, count, memory hash.

OPEN: on signed-overflow operands `add` panics. The oracle returns success (result 0) at
instruction 456, while the emulator (the kernel's step code) continues into the panic
path and reaches the WASI fd_write import at instruction 1022; both agree bit for bit
(status, count, memory hash) up to instruction 455 under every cost limit. The panic
message is printed through fd_write by the reference, so the oracle is the suspect; the
strict xfail below records the divergence until it is resolved."""
import numpy as np
import pytest

import oracle_py as O
from conftest import golden
from helpers import compare, emu_run, gpu_run

I32 = 0x7F


def _s32(x):
    return x - (1 << 32) if x >> 31 else x


def _overflows(a, b):
    return not -(1 << 31) <= _s32(a) + _s32(b) < (1 << 31)


def _rows(n, seed):
    """Operands whose i32 sum does not overflow (edges included)."""
    rng = np.random.default_rng(seed)
    v = rng.integers(0, 1 << 32, size=(n, 2), dtype=np.uint64)
    v[::7] = [0x7FFFFFFF, 0]
    v[3::7] = [0x80000000, 0x7FFFFFFF]
    v[1::5] = [2, 2]
    return [[int(a), int(b)] for a, b in v if not _overflows(int(a), int(b))]


def _oracle(rows):
    O.set_lazy_imports(True)
    try:
        m = O.Module(golden("rust_add.wasm"))
        return [O.Instance(m).invoke("add", r) for r in rows]
    finally:
        O.set_lazy_imports(False)


def test_rust_add_oracle_kat():
    code, vals, cnt, _ = _oracle([[2, 2]])[0]
    assert (code, vals) == (0, [4])


def test_rust_add_emulator():
    rows = _rows(64, 1)
    ref = _oracle(rows)
    got = emu_run(golden("rust_add.wasm"), "add", rows, [I32, I32], [I32])
    assert compare(ref, *got, [I32]) == []


@pytest.mark.gpu
def test_gpu_rust_add(built):
    rows = _rows(2048, 2)
    ref = _oracle(rows)
    got = gpu_run(golden("rust_add.wasm"), "add", rows, [I32, I32], [I32], device=0)
    assert compare(ref, *got, [I32]) == []
    assert got[0][1] == [4]


@pytest.mark.xfail(strict=True, reason="open oracle/emulator divergence on the panic path")
def test_rust_add_overflow_panic_path():
    rows = [[0x7FFFFFFF, 5], [1070428841, 1339305888]]
    ref = _oracle(rows)
    got = emu_run(golden("rust_add.wasm"), "add", rows, [I32, I32], [I32])
    assert compare(ref, *got, [I32]) == []
