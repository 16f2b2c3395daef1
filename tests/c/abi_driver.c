/* A plain C caller of the batched ABI (include/wasmedge_batch.h) -- what a reference-side
 * embedder would write: no Python, no ctypes. Runs fibonacci.wasm's `fib`
 * on N instances (n = i mod 25) through BatchCreate / Execute / Results, the staged
 * SetArgs / Reset / Run path and MemoryHash, over one device and over two shards
 * (Devices = {0, 0}), and checks every result, status and instruction count against fib
 * and the reference's counting rule (fib(n) retires 15 instructions per internal call and
 * 6 per leaf: tests/test_kat.py). Prints one line per check; exit status 0 = all passed.
 * Built by wasmedge_amd/csrc/Makefile; run by tests/test_abi.py on the GPU. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "wasmedge_batch.h"

static uint64_t fib(uint32_t n) { return n < 2 ? 1 : fib(n - 1) + fib(n - 2); }
static uint64_t calls(uint32_t n) { return n < 2 ? 1 : 1 + calls(n - 1) + calls(n - 2); }
static uint64_t instrs(uint32_t n) {   /* leaves L = (calls + 1) / 2, internal I = L - 1 */
  const uint64_t c = calls(n), leaves = (c + 1) / 2;
  return 6 * leaves + 15 * (c - leaves);
}

static int check(const char *what, const WasmEdge_BatchConfigure *conf, const uint8_t *wasm,
                 uint32_t len, uint32_t n) {
  WasmEdge_Result res;
  WasmEdge_BatchContext *B = WasmEdge_BatchCreate(conf, wasm, len, n, &res);
  if (!B) {
    printf("%s: create failed 0x%02x %s\n", what, res.Code, WasmEdge_BatchGetLastError(NULL));
    return 1;
  }
  WasmEdge_Value *params = calloc(n, sizeof(WasmEdge_Value)), *rets = calloc(n, sizeof(WasmEdge_Value));
  uint8_t *st = calloc(n, 1);
  uint64_t *cnt = calloc(n, 8), *hash = calloc(n, 8);
  for (uint32_t i = 0; i < n; i++) {
    params[i].Value = i % 25;
    params[i].Type = WasmEdge_ValType_I32;
  }
  WasmEdge_String fn = {3, "fib"};
  int bad = 0;
  for (int pass = 0; pass < 3 && !bad; pass++) {
    if (pass == 0) {
      res = WasmEdge_BatchExecute(B, fn, params, 1, rets, 1, st, cnt);
    } else if (pass == 2) {   /* SURVEY 8(b)'s form: a WasmEdge_Result per instance */
      WasmEdge_Result *pr = calloc(n, sizeof(WasmEdge_Result));
      res = WasmEdge_BatchReset(B, NULL);
      if (!res.Code) res = WasmEdge_BatchExecuteResults(B, fn, params, 1, rets, 1, pr, cnt);
      for (uint32_t i = 0; i < n; i++) st[i] = pr[i].Code;
      free(pr);
    } else {   /* the staged form, as the bench drives it */
      double ks = 0;
      res = WasmEdge_BatchSetArgs(B, fn, params, 1);
      if (!res.Code) res = WasmEdge_BatchReset(B, NULL);
      if (!res.Code) res = WasmEdge_BatchRun(B, &ks);
      if (!res.Code) res = WasmEdge_BatchResults(B, rets, 1, st, cnt);
      if (!res.Code && !(ks > 0)) bad = 1;
    }
    if (res.Code) {
      printf("%s: pass %d failed 0x%02x %s\n", what, pass, res.Code, WasmEdge_BatchGetLastError(B));
      bad = 1;
      break;
    }
    for (uint32_t i = 0; i < n && !bad; i++)
      if (st[i] || (uint32_t)rets[i].Value != (uint32_t)fib(i % 25) || rets[i].Type != WasmEdge_ValType_I32 ||
          cnt[i] != instrs(i % 25)) {
        printf("%s: instance %u: status 0x%02x value %u count %llu (want %llu, %llu)\n", what, i, st[i],
               (unsigned)rets[i].Value, (unsigned long long)cnt[i], (unsigned long long)fib(i % 25),
               (unsigned long long)instrs(i % 25));
        bad = 1;
      }
  }
  /* fibonacci.wasm has no memory: every hash is the hash of 0 pages, the same for all */
  if (!bad && (res = WasmEdge_BatchMemoryHash(B, hash)).Code) bad = 1;
  for (uint32_t i = 1; i < n && !bad; i++)
    if (hash[i] != hash[0]) bad = 1;
  if (!bad && WasmEdge_BatchGetInstanceCount(B) != n) bad = 1;
  if (!bad && WasmEdge_BatchExecute(B, (WasmEdge_String){4, "nope"}, params, 1, rets, 1, st, cnt).Code != 0x05)
    bad = 1;   /* FuncNotFound */
  printf("%s: %u instances %s\n", what, n, bad ? "FAILED" : "ok");
  WasmEdge_BatchDelete(B);
  free(params); free(rets); free(st); free(cnt); free(hash);
  return bad;
}

int main(int argc, char **argv) {
  if (argc < 2) { fprintf(stderr, "usage: abi_driver fibonacci.wasm\n"); return 2; }
  FILE *f = fopen(argv[1], "rb");
  if (!f) { perror(argv[1]); return 2; }
  uint8_t buf[4096];
  const uint32_t len = (uint32_t)fread(buf, 1, sizeof buf, f);
  fclose(f);
  printf("build %s\n", WasmEdge_BatchGetBuildHash());
  WasmEdge_BatchConfigure one;
  memset(&one, 0, sizeof one);
  one.DeviceOrdinal = 0;
  int bad = check("one device", &one, buf, len, 1000);
  WasmEdge_BatchConfigure two = one;
  const int32_t devs[2] = {0, 0};
  two.Devices = devs;
  two.DeviceCount = 2;
  two.Partition = WASMEDGE_BATCH_PARTITION_INTERLEAVE;
  bad |= check("two shards", &two, buf, len, 1000);
  return bad;
}
