// dbc.h -- the device bytecode (DBC) shared by the host lowering (lower.cpp) and the
// CDNA4 interpreter kernel (batch_kernel.hip).
//
// The reference executes AST::Instruction records (32 B each, include/ast/instruction.h:
// 27-274) on a std::vector<ValVariant> stack (include/runtime/stackmgr.h).  The DBC is
// a REGISTER form of the same program: every operand-stack position, local and global
// has a fixed 32-bit "cell" index known at lowering time (the validator already knows
// every stack height, lib/validator/formchecker.cpp), so an instruction names its
// source/destination cells instead of pushing/popping.  local.get/const/nop/block/loop/
// end/reinterpret are folded away; `cnt` keeps the reference's instruction count exact
// (engine.cpp:1618-1621 counts every dispatched wasm instruction, a13 in SURVEY.md).
//
// Encoding: 16 bytes, one s_load_dwordx4 per dispatch.
//   w0: op (bits 0-15) | cnt (16-23: wasm instrs retired by this dispatch) |
//       post (24-30: trailing folded instrs not counted when this instruction traps) |
//       bit 31 = CTL: the op may branch, call, return or trap (the kernel re-checks
//       wave convergence only after such ops)
//   w1: a (0-15) | b (16-31)       source cells / counts
//   w2: c (0-15) | d (16-31)       destination cell / extra (d = signed tcnt on branches)
//   w3: imm                        immediate / branch target / memarg offset
#pragma once
#include <stdint.h>

#define WB_TCODE_DONE 0x100u    // internal: the lane returned from its entry function
#define DBC_CTL 0x80000000u      // w0 flag: control transfer / trap possible
#define DBC_EXIT_PC 0xFFFFFu      // 20-bit return-pc field value that ends the lane
#define DBC_MAX_PC 0xFFFF0u
#define DBC_CELL_BYTES 4

struct DInstr {
  uint32_t w0, w1, w2, w3;
};

// X-macro list of device ops. Field use is documented per group.
#define DBC_OPS(X)                                                                     \
  /* control: imm = target pc, d = tcnt (signed, added when taken) */                 \
  X(NOP_CNT) X(JMP) X(BR_IF) X(BR_UNLESS) X(BR_IF_MOV1) X(BR_IF_MOV2)                 \
  /* fused compare-and-branch: taken when (a CMP b); _I: b field is a signed imm16     */ \
  X(BR_EQ) X(BR_NE) X(BR_LT_S) X(BR_LT_U) X(BR_GT_S) X(BR_GT_U) X(BR_LE_S) X(BR_LE_U)   \
  X(BR_GE_S) X(BR_GE_U)                                                                \
  X(BR_EQ_I) X(BR_NE_I) X(BR_LT_S_I) X(BR_LT_U_I) X(BR_GT_S_I) X(BR_GT_U_I) X(BR_LE_S_I)\
  X(BR_LE_U_I) X(BR_GE_S_I) X(BR_GE_U_I)                                               \
  X(BR_TABLE)     /* a = index cell, b = #labels-1, imm = brtab offset              */ \
  X(CALL)         /* a = L (caller live cells), b = arg cells, c = local cells       */ \
  X(CALL_INDIRECT)/* a = L, b = arg cells, c = index cell, d = table, imm = type id  */ \
  X(RET)          /* a = first result cell, b = result cells                         */ \
  X(POST_CALL)    /* a = L                                                           */ \
  X(ZERO_LOCALS)  /* a = first cell, b = count                                       */ \
  X(UNREACHABLE)                                                                       \
  X(HOST_CALL)    /* a = first arg cell (results land there), b = arg cells,         */ \
                  /* c = result cells, imm = function index of the import            */ \
  X(TAIL_CALL)    /* return_call: a = L, b = arg cells, c = local cells, imm = target */ \
  X(TAIL_CALL_INDIRECT) /* return_call_indirect: fields as CALL_INDIRECT             */ \
  /* data movement: a -> c ; d = cond cell for select                                 */ \
  X(MOV32) X(MOV64) X(MOV128) X(CONST32) X(CONST64) X(CONST128)                       \
  X(SELECT32) X(SELECT64) X(SELECT128)                                                 \
  /* memory: a = address cell, b = value cell (store), c = dst, imm = offset          */ \
  X(LD8S32) X(LD8U32) X(LD16S32) X(LD16U32) X(LD32)                                    \
  X(LD8S64) X(LD8U64) X(LD16S64) X(LD16U64) X(LD32S64) X(LD32U64) X(LD64) X(LD128)     \
  X(ST8) X(ST16) X(ST32) X(ST64) X(ST128)                                               \
  X(MEM_SIZE) X(MEM_GROW) X(MEM_FILL) X(MEM_COPY) X(MEM_INIT) X(DATA_DROP)             \
  X(TABLE_GET)    /* a = index cell, c = dst, d = table                              */ \
  X(TABLE_SET)    /* a = index cell, b = ref cell, d = table (per-lane tables)       */ \
  X(TABLE_SIZE)   /* c = dst, d = table                                              */ \
  X(TABLE_GROW)   /* a = init ref cell, b = n cell, c = dst, d = table               */ \
  X(TABLE_FILL)   /* a = dst idx cell, b = ref cell, c = n cell, imm = table         */ \
  X(TABLE_COPY)   /* a = dst idx, b = src idx, c = n, imm = dst table | src table<<16 */ \
  X(TABLE_INIT)   /* a = dst idx, b = src idx, c = n, imm = table | elem seg<<16     */ \
  X(ELEM_DROP)    /* imm = elem segment                                              */ \
  /* i32 binary: c = a op b ; *_I: c = a op imm                                       */ \
  X(I32_ADD) X(I32_SUB) X(I32_MUL) X(I32_DIV_S) X(I32_DIV_U) X(I32_REM_S) X(I32_REM_U) \
  X(I32_AND) X(I32_OR) X(I32_XOR) X(I32_SHL) X(I32_SHR_S) X(I32_SHR_U) X(I32_ROTL)     \
  X(I32_ROTR) X(I32_EQ) X(I32_NE) X(I32_LT_S) X(I32_LT_U) X(I32_GT_S) X(I32_GT_U)      \
  X(I32_LE_S) X(I32_LE_U) X(I32_GE_S) X(I32_GE_U)                                      \
  X(I32_ADD_I) X(I32_SUB_I) X(I32_MUL_I) X(I32_DIV_S_I) X(I32_DIV_U_I) X(I32_REM_S_I)  \
  X(I32_REM_U_I) X(I32_AND_I) X(I32_OR_I) X(I32_XOR_I) X(I32_SHL_I) X(I32_SHR_S_I)     \
  X(I32_SHR_U_I) X(I32_ROTL_I) X(I32_ROTR_I) X(I32_EQ_I) X(I32_NE_I) X(I32_LT_S_I)     \
  X(I32_LT_U_I) X(I32_GT_S_I) X(I32_GT_U_I) X(I32_LE_S_I) X(I32_LE_U_I) X(I32_GE_S_I)  \
  X(I32_GE_U_I)                                                                        \
  X(I32_EQZ) X(I32_CLZ) X(I32_CTZ) X(I32_POPCNT) X(I32_EXT8S) X(I32_EXT16S)            \
  /* superinstructions: c = a + b + d ; c = rot(a ^ b, imm)                           */ \
  X(I32_ADD3) X(I32_XOR_ROTR_I) X(I32_XOR_ROTL_I)                                      \
  /* ARX pairs (peephole, see frontend.cpp fuse_arx): c = a + b (+ d);                 */ \
  /*   ADD_XROTR_I:  d = rotr(d ^ c, imm)                                             */ \
  /*   ADD3_XROTR_I: y = rotr(y ^ c, imm >> 16), y = imm & 0xFFFF                      */ \
  X(I32_ADD_XROTR_I) X(I32_ADD3_XROTR_I)                                               \
  /* i64 binary (compares write an i32 cell)                                          */ \
  X(I64_ADD) X(I64_SUB) X(I64_MUL) X(I64_DIV_S) X(I64_DIV_U) X(I64_REM_S) X(I64_REM_U) \
  X(I64_AND) X(I64_OR) X(I64_XOR) X(I64_SHL) X(I64_SHR_S) X(I64_SHR_U) X(I64_ROTL)     \
  X(I64_ROTR) X(I64_EQ) X(I64_NE) X(I64_LT_S) X(I64_LT_U) X(I64_GT_S) X(I64_GT_U)      \
  X(I64_LE_S) X(I64_LE_U) X(I64_GE_S) X(I64_GE_U)                                      \
  /* *_I: b-operand is imm sign-extended to 64 bits                                   */ \
  X(I64_ADD_I) X(I64_SUB_I) X(I64_MUL_I) X(I64_DIV_S_I) X(I64_DIV_U_I) X(I64_REM_S_I)  \
  X(I64_REM_U_I) X(I64_AND_I) X(I64_OR_I) X(I64_XOR_I) X(I64_SHL_I) X(I64_SHR_S_I)     \
  X(I64_SHR_U_I) X(I64_ROTL_I) X(I64_ROTR_I) X(I64_EQ_I) X(I64_NE_I) X(I64_LT_S_I)     \
  X(I64_LT_U_I) X(I64_GT_S_I) X(I64_GT_U_I) X(I64_LE_S_I) X(I64_LE_U_I) X(I64_GE_S_I)  \
  X(I64_GE_U_I)                                                                        \
  X(I64_EQZ) X(I64_CLZ) X(I64_CTZ) X(I64_POPCNT) X(I64_EXT8S) X(I64_EXT16S)            \
  X(I64_EXT32S) X(I64_EXTEND_I32_S) X(I64_EXTEND_I32_U)                                \
  /* floating point                                                                   */ \
  X(F32_ADD) X(F32_SUB) X(F32_MUL) X(F32_DIV) X(F32_MIN) X(F32_MAX) X(F32_COPYSIGN)    \
  X(F32_EQ) X(F32_NE) X(F32_LT) X(F32_GT) X(F32_LE) X(F32_GE)                          \
  X(F32_ABS) X(F32_NEG) X(F32_CEIL) X(F32_FLOOR) X(F32_TRUNC) X(F32_NEAREST) X(F32_SQRT)\
  X(F64_ADD) X(F64_SUB) X(F64_MUL) X(F64_DIV) X(F64_MIN) X(F64_MAX) X(F64_COPYSIGN)    \
  X(F64_EQ) X(F64_NE) X(F64_LT) X(F64_GT) X(F64_LE) X(F64_GE)                          \
  X(F64_ABS) X(F64_NEG) X(F64_CEIL) X(F64_FLOOR) X(F64_TRUNC) X(F64_NEAREST) X(F64_SQRT)\
  /* conversions: a -> c                                                              */ \
  X(I32_TRUNC_F32_S) X(I32_TRUNC_F32_U) X(I32_TRUNC_F64_S) X(I32_TRUNC_F64_U)          \
  X(I64_TRUNC_F32_S) X(I64_TRUNC_F32_U) X(I64_TRUNC_F64_S) X(I64_TRUNC_F64_U)          \
  X(I32_TRUNC_SAT_F32_S) X(I32_TRUNC_SAT_F32_U) X(I32_TRUNC_SAT_F64_S)                 \
  X(I32_TRUNC_SAT_F64_U) X(I64_TRUNC_SAT_F32_S) X(I64_TRUNC_SAT_F32_U)                 \
  X(I64_TRUNC_SAT_F64_S) X(I64_TRUNC_SAT_F64_U)                                        \
  X(F32_CONVERT_I32_S) X(F32_CONVERT_I32_U) X(F32_CONVERT_I64_S) X(F32_CONVERT_I64_U)  \
  X(F64_CONVERT_I32_S) X(F64_CONVERT_I32_U) X(F64_CONVERT_I64_S) X(F64_CONVERT_I64_U)  \
  X(F32_DEMOTE_F64) X(F64_PROMOTE_F32)                                                 \
  /* SIMD128 (4 cells per value): c = a op b, or a op (i32 cell b)                    */ \
  X(V_NOT) X(V_AND) X(V_ANDNOT) X(V_OR) X(V_XOR) X(V_BITSELECT) X(V_ANY_TRUE)          \
  X(V_I8X16_SPLAT) X(V_I16X8_SPLAT) X(V_I32X4_SPLAT) X(V_I64X2_SPLAT)                  \
  X(V_EXTRACT32) X(V_EXTRACT64) X(V_REPLACE32) X(V_REPLACE64)                          \
  X(V_EXTRACT8S) X(V_EXTRACT8U) X(V_EXTRACT16S) X(V_EXTRACT16U) X(V_REPLACE8)          \
  X(V_REPLACE16) X(V_SHUFFLE) X(V_SWIZZLE)                                             \
  X(V_I8X16_ADD) X(V_I8X16_SUB) X(V_I16X8_ADD) X(V_I16X8_SUB) X(V_I16X8_MUL)           \
  X(V_I32X4_ADD) X(V_I32X4_SUB) X(V_I32X4_MUL) X(V_I64X2_ADD) X(V_I64X2_SUB)           \
  X(V_I64X2_MUL) X(V_I8X16_EQ) X(V_I8X16_NE) X(V_I16X8_EQ) X(V_I16X8_NE)               \
  X(V_I32X4_EQ) X(V_I32X4_NE) X(V_I32X4_LT_S) X(V_I32X4_LT_U) X(V_I32X4_GT_S)          \
  X(V_I32X4_GT_U) X(V_I32X4_LE_S) X(V_I32X4_LE_U) X(V_I32X4_GE_S) X(V_I32X4_GE_U)      \
  X(V_I64X2_EQ) X(V_I64X2_NE) X(V_I64X2_LT_S) X(V_I64X2_GT_S) X(V_I64X2_LE_S)          \
  X(V_I64X2_GE_S)                                                                      \
  X(V_I8X16_SHL) X(V_I8X16_SHR_S) X(V_I8X16_SHR_U) X(V_I16X8_SHL) X(V_I16X8_SHR_S)     \
  X(V_I16X8_SHR_U) X(V_I32X4_SHL) X(V_I32X4_SHR_S) X(V_I32X4_SHR_U) X(V_I64X2_SHL)     \
  X(V_I64X2_SHR_S) X(V_I64X2_SHR_U)                                                    \
  X(V_I8X16_ALL_TRUE) X(V_I16X8_ALL_TRUE) X(V_I32X4_ALL_TRUE) X(V_I64X2_ALL_TRUE)      \
  X(V_I8X16_BITMASK) X(V_I16X8_BITMASK) X(V_I32X4_BITMASK) X(V_I64X2_BITMASK)          \
  X(V_I32X4_NEG) X(V_I64X2_NEG) X(V_I32X4_ABS) X(V_I64X2_ABS)                          \
  X(V_F32X4_ADD) X(V_F32X4_SUB) X(V_F32X4_MUL) X(V_F32X4_DIV) X(V_F32X4_MIN)           \
  X(V_F32X4_MAX) X(V_F32X4_PMIN) X(V_F32X4_PMAX) X(V_F32X4_EQ) X(V_F32X4_NE)           \
  X(V_F32X4_LT) X(V_F32X4_GT) X(V_F32X4_LE) X(V_F32X4_GE) X(V_F32X4_ABS)               \
  X(V_F32X4_NEG) X(V_F32X4_SQRT)                                                       \
  X(V_F64X2_ADD) X(V_F64X2_SUB) X(V_F64X2_MUL) X(V_F64X2_DIV) X(V_F64X2_MIN)           \
  X(V_F64X2_MAX) X(V_F64X2_PMIN) X(V_F64X2_PMAX) X(V_F64X2_EQ) X(V_F64X2_NE)           \
  X(V_F64X2_LT) X(V_F64X2_GT) X(V_F64X2_LE) X(V_F64X2_GE) X(V_F64X2_ABS)               \
  X(V_F64X2_NEG) X(V_F64X2_SQRT)                                                       \
  X(V_F32X4_SPLAT) X(V_F64X2_SPLAT)                                                    \
  X(V_LD8X8S) X(V_LD8X8U) X(V_LD16X4S) X(V_LD16X4U) X(V_LD32X2S) X(V_LD32X2U)          \
  X(V_LD8SPLAT) X(V_LD16SPLAT) X(V_LD32SPLAT) X(V_LD64SPLAT) X(V_LD32ZERO)             \
  X(V_LD64ZERO)                                                                        \
  /* generic lane-wise ops, imm = the 0xFD sub-opcode: c = op(a, b) / c = op(a)        */ \
  X(V_BINX) X(V_UNX)                                                                   \
  /* a = address cell, b = vector cell, c = dst, d = lane | log2(bytes) << 8, imm = off */ \
  X(V_LDLANE) X(V_STLANE)                                                              \
  /* memories past the first (MultiMemories; the per-lane step only), k = memory index:  */ \
  /*   XLD: a = address, b = k, c = dst, d = the memory-0 load op, imm = offset          */ \
  /*   XST: a = address, b = value, c = k, d = the memory-0 store op, imm = offset       */ \
  /*   XLANE: as V_LDLANE / V_STLANE, d = lane | log2(bytes) << 4 | load << 6 | k << 8   */ \
  /*   XMEM_SIZE: b = k, c = dst; XMEM_GROW: a = pages, b = k, c = dst                    */ \
  /*   XMEM_FILL: a, b, c as MEM_FILL, imm = k; XMEM_INIT: as MEM_INIT, d = k            */ \
  /*   XMEM_COPY: as MEM_COPY, imm = dst memory | src memory << 16 (one of them > 0)    */ \
  X(XLD) X(XST) X(XLANE) X(XMEM_SIZE) X(XMEM_GROW) X(XMEM_FILL) X(XMEM_COPY) X(XMEM_INIT)  \
  X(DBC_NUM_OPS)

enum DOp : uint16_t {
#define DBC_ENUM(n) OP_##n,
  DBC_OPS(DBC_ENUM)
#undef DBC_ENUM
};

// Per-function info table (device): used by call_indirect.
struct DFunc {
  uint32_t entry_pc;   // first instruction (the ZERO_LOCALS prologue when it has locals)
  uint32_t type_id;    // canonical structural function-type id
};

// Batch status codes beyond the reference ErrCodes (include/common/enum.inc:573-749).
#define WB_STATUS_RUNNING 0xFFu
#define WB_STATUS_OK 0x00u
#define WB_ERR_INTERRUPTED 0x07u        // ErrCode::Interrupted (fuel / time limit)
#define WB_ERR_STACK_EXHAUSTED 0xB0u    // device call stack full (no reference code)
#define WB_ERR_HOST_CALL 0xB1u          // lane yielded at a host import; BatchRun's host loop
                                        // services it and resumes the lane. It stays the
                                        // final status only when no host function is
                                        // registered for that import.
// The import index a lane parks with when its memory.grow needs pool rows the host has not
// allocated yet (KParams::grow_host): the host allocates them and completes the grow.
#define WB_GROW_CALL 0xFFFFFFFEu
// ... when a call would pass the call stack's reserved cells while the stack may still grow
// (KParams::gs_grow): the host grows it and the lane runs the call again (hostcall.cpp
// grow_stack)
#define WB_STACK_CALL 0xFFFFFFFDu
// ... | t when a table.grow would pass table t's per-lane capacity while tables may still
// widen (KParams::tg_grow; t < 2^24): the host widens every lane's table t and the lane runs
// the grow again (hostcall.cpp widen_tables)
#define WB_TGROW_CALL 0xF0000000u
#define WB_TGROW_MASK 0xFF000000u
