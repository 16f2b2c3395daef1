"""Regenerate tests/golden/ fixtures from the reference's own test data (run in the
build container, where /root/reference exists; the GPU box only reads the outputs).

Fixtures are data only (wasm binaries the reference's tests hold, and their expected
answers):
  mt19937.wasm      bytes of test/thread/ThreadTest.cpp:31-150 (MersenneTwister19937)
  mt19937.json      answers test/thread/ThreadTest.cpp:152-157, args :168-169
  fibonacci.wasm    tools/wasmedge/examples/fibonacci.wasm (README: fib 8 -> 34)
  factorial.wasm    tools/wasmedge/examples/factorial.wasm (README: fac 12 -> 479001600)
  apitest.wasm      test/api/apiTestData/test.wasm
  externref_funcs.wasm  test/externref/externrefTestData/funcs.wasm
                    (answers in test/externref/ExternrefTest.cpp:308-356)
  externref_stl.wasm    test/externref/externrefTestData/stl.wasm (:372-465)
  rust_add.wasm     tools/wasmedge/examples/add.wasm (compiled Rust/WASI; add 2 2 -> 4)
  hello.wasm        tools/wasmedge/examples/hello.wasm (compiled Rust/WASI command;
                    README.md:5-15 runs it as `wasmedge hello.wasm 1 2 3`)
  qjs.wasm          tools/wasmedge/examples/js/qjs.wasm (QuickJS, a WASI command;
                    js/README.md:9-14 runs `wasmedge --dir .:. qjs.wasm hello.js 1 2 3`)
  executor_interrupt.wasm  bytes of test/executor/ExecutorTest.cpp:122-126 (endless
                    loop in _start; cancel -> Interrupted, :127-145)
"""
import json
import os
import re
import shutil
import sys

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    src = open(os.path.join(REF, "test/thread/ThreadTest.cpp")).read()
    m = re.search(r"MersenneTwister19937\{(.*?)\};", src, re.S)
    data = bytes(int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]{2}", m.group(1)))
    assert len(data) == 1481, len(data)
    open(os.path.join(OUT, "mt19937.wasm"), "wb").write(data)
    a = re.search(r"Answers\{(.*?)\};", src, re.S)
    answers = [int(x) for x in re.findall(r"UINT64_C\((\d+)\)", a.group(1))]
    json.dump({"source": "test/thread/ThreadTest.cpp:31-163",
               "func": "mt19937",
               "args": [[2504 * i, 5489, 100000 + i] for i in range(len(answers))],
               "answers": answers}, open(os.path.join(OUT, "mt19937.json"), "w"), indent=1)
    for name in ("fibonacci", "factorial"):
        shutil.copy(os.path.join(REF, "tools/wasmedge/examples/%s.wasm" % name),
                    os.path.join(OUT, name + ".wasm"))
    shutil.copy(os.path.join(REF, "test/api/apiTestData/test.wasm"),
                os.path.join(OUT, "apitest.wasm"))
    shutil.copy(os.path.join(REF, "test/externref/externrefTestData/funcs.wasm"),
                os.path.join(OUT, "externref_funcs.wasm"))
    shutil.copy(os.path.join(REF, "test/externref/externrefTestData/stl.wasm"),
                os.path.join(OUT, "externref_stl.wasm"))
    shutil.copy(os.path.join(REF, "tools/wasmedge/examples/add.wasm"),
                os.path.join(OUT, "rust_add.wasm"))
    shutil.copy(os.path.join(REF, "tools/wasmedge/examples/hello.wasm"),
                os.path.join(OUT, "hello.wasm"))
    shutil.copy(os.path.join(REF, "tools/wasmedge/examples/js/qjs.wasm"),
                os.path.join(OUT, "qjs.wasm"))
    src = open(os.path.join(REF, "test/executor/ExecutorTest.cpp")).read()
    m = re.search(r"std::array<WasmEdge::Byte, 46> Wasm\{(.*?)\};", src, re.S)
    data = bytes(int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]{2}", m.group(1)))
    assert len(data) == 46, len(data)
    open(os.path.join(OUT, "executor_interrupt.wasm"), "wb").write(data)
    print("ok", len(answers))


if __name__ == "__main__":
    sys.exit(main())
