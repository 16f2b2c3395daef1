"""A compiled Rust/WASI module from the reference (tools/wasmedge/examples/add.wasm,
fixture tests/golden/rust_add.wasm, 1.7 MB): the loader, validator and lowering over a
real toolchain's output (hundreds of functions, WASI imports that `add` never reaches on
non-overflowing operands). Known answer: `wasmedge --reactor add.wasm add 2 2` -> 4
(docs/book/en/src/extend/build_for_android.md:70-71). Per-lane operands are checked
against the oracle: status, result, count, memory hash.

Overflowing operands take the panic path: `add` runs 3,725 instructions and then calls
the WASI import fd_write to print the panic message. The oracle and the kernel's step code
agree bit for bit on that path (status, count, memory hash) under every cost limit. Two
bugs hid this in round 1. The oracle stopped the entry function at the first instruction
of the next function (see tests/test_entry_layout.py). The two sides also ran with
different page budgets: the emulator allowed the module's initial 17 pages, the oracle 65536,
so the panic handler's memory.grow at instruction 687 differed."""
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
    """Non-overflowing operands return; overflowing ones (every 3rd row) take the panic
    path to the fd_write import (0xB1, no host function bound here) at the oracle's count
    with the oracle's memory."""
    rows = _rows(2048, 2)
    ov = [[0x7FFFFFFF, 1 + k] if k % 2 else [0x80000000, 0xFFFFFFFF - k] for k in range(len(rows[::3]))]
    rows[::3] = ov
    O.set_lazy_imports(True)
    try:
        m = O.Module(golden("rust_add.wasm"), page_limit=32)
        ref = [O.Instance(m).invoke("add", r) for r in rows]
    finally:
        O.set_lazy_imports(False)
    ref = [(0xB1 if c == 0x8D else c, v, n, h) for c, v, n, h in ref]
    got = gpu_run(golden("rust_add.wasm"), "add", rows, [I32, I32], [I32], device=0,
                  max_memory_page=32)
    assert compare(ref, *got, [I32]) == []
    assert rows[1] == [2, 2] and got[0][1] == [4]
    assert sum(1 for r in ref if r[0] == 0xB1) == len(ov)


def test_rust_add_overflow_panic_path():
    """Panic path up to the fd_write import, with matched page budgets: the oracle (no
    host function bound: HostFuncFailed 0x8D) and the emulator (import reached: 0xB1)
    stop at the same instruction with the same memory; every cost limit on the way gives
    the same CostLimitExceeded state on both."""
    rows = [[0x7FFFFFFF, 5], [1070428841, 1339305888]]
    O.set_lazy_imports(True)
    try:
        m = O.Module(golden("rust_add.wasm"), page_limit=32)
        for lim in (0, 456, 687, 1022, 2000, 3724, 3725):
            ref = [O.Instance(m, cost_limit=lim).invoke("add", r) for r in rows]
            _, st, cnt, h = emu_run(golden("rust_add.wasm"), "add", rows, [I32, I32], [I32],
                                    max_pages=32, cost_limit=lim)
            for i, (code, _v, c, oh) in enumerate(ref):
                want = 0xB1 if code == 0x8D else code
                assert (int(st[i]), int(cnt[i]), int(h[i])) == (want, c, oh), (lim, i)
                if lim == 0:
                    assert (code, c) == (0x8D, 3725)
    finally:
        O.set_lazy_imports(False)
