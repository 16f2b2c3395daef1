"""Minimal WebAssembly text-format assembler (WAT -> .wasm bytes).

This image has no wat2wasm/emcc/rustc, so the config modules (BASELINE.json configs 2-5)
and the parity micro-modules are authored in WAT and assembled here.  Supports the subset
of the text format the build's modules use: module fields (type, import func, func,
table, memory, global, export, start, elem, data), inline exports, $names, flat and folded
instructions, block types via (param ..)(result ..) or (type N), and all opcodes in
`opcodes.py`.  It is checked against the reference's own .wat/.wasm pairs in
tests/test_wat.py (tools/wasmedge/examples/{fibonacci,factorial}).
"""
import math
import re
import struct

from .opcodes import OPS, ALIASES, VALTYPES
from . import opcodes as O


# ---------------------------------------------------------------- s-expressions
_TOK = re.compile(r'\s+|;;[^\n]*|\(;.*?;\)|(\()|(\))|("(?:[^"\\]|\\.)*")|([^\s()";]+)', re.S)


def _tokenize(src):
    out = []
    pos = 0
    while pos < len(src):
        m = _TOK.match(src, pos)
        if not m:
            raise SyntaxError("bad token at %d: %r" % (pos, src[pos:pos + 20]))
        pos = m.end()
        if m.group(1):
            out.append("(")
        elif m.group(2):
            out.append(")")
        elif m.group(3):
            out.append(Str(m.group(3)))
        elif m.group(4):
            out.append(m.group(4))
    return out


class Str(str):
    """A quoted string token (kept distinct from atoms)."""


def _parse(tokens):
    stack = [[]]
    for t in tokens:
        if t == "(":
            stack.append([])
        elif t == ")":
            x = stack.pop()
            stack[-1].append(x)
        else:
            stack[-1].append(t)
    if len(stack) != 1:
        raise SyntaxError("unbalanced parens")
    return stack[0]


def _strbytes(s):
    body = s[1:-1]
    out = bytearray()
    i = 0
    while i < len(body):
        c = body[i]
        if c == "\\":
            n = body[i + 1]
            esc = {"n": 10, "t": 9, "r": 13, '"': 34, "'": 39, "\\": 92}
            if n in esc:
                out.append(esc[n])
                i += 2
            elif n == "u":
                j = body.index("}", i)
                out += chr(int(body[i + 3:j], 16)).encode()
                i = j + 1
            else:
                out.append(int(body[i + 1:i + 3], 16))
                i += 3
        else:
            out += c.encode()
            i += 1
    return bytes(out)


# ---------------------------------------------------------------- encoders
def uleb(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def sleb(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if (v == 0 and not b & 0x40) or (v == -1 and b & 0x40):
            out.append(b)
            return bytes(out)
        out.append(b | 0x80)


def _vec(items):
    return uleb(len(items)) + b"".join(items)


def _name(s):
    b = s.encode() if not isinstance(s, bytes) else s
    return uleb(len(b)) + b


def parse_int(tok, bits):
    t = tok.replace("_", "")
    neg = t.startswith("-")
    if t[0] in "+-":
        t = t[1:]
    v = int(t, 16) if t.startswith("0x") else int(t)
    if neg:
        v = -v
    v &= (1 << bits) - 1
    if v >= 1 << (bits - 1):
        v -= 1 << bits
    return v


def _float_bits(tok, bits):
    t = tok.replace("_", "")
    sign = 0
    if t[0] in "+-":
        sign = 1 if t[0] == "-" else 0
        t = t[1:]
    ebits, mbits = (8, 23) if bits == 32 else (11, 52)
    if t == "inf":
        v = ((1 << ebits) - 1) << mbits
    elif t.startswith("nan"):
        payload = int(t[6:], 16) if t.startswith("nan:0x") else 1 << (mbits - 1)
        v = (((1 << ebits) - 1) << mbits) | payload
    else:
        if t.startswith("0x"):
            f = float.fromhex(t)
        else:
            f = float(t)
        if bits == 32:
            v = struct.unpack("<I", struct.pack("<f", f))[0]
        else:
            v = struct.unpack("<Q", struct.pack("<d", f))[0]
        v &= ~(1 << (bits - 1))
    return v | (sign << (bits - 1))


# ---------------------------------------------------------------- module builder
class _Func:
    def __init__(self):
        self.name = None
        self.typeidx = None
        self.params = []
        self.results = []
        self.locals = []
        self.local_names = {}
        self.body = []
        self.exports = []
        self.imported = None


class Assembler:
    def __init__(self, sexpr):
        self.types = []          # list of (params tuple, results tuple)
        self.type_names = {}
        self.funcs = []          # imports first
        self.func_names = {}
        self.tables = []         # (reftype, min, max)
        self.table_names = {}
        self.mems = []           # (min, max)
        self.mem_names = {}
        self.globals = []        # (valtype, mut, init bytes)
        self.global_names = {}
        self.exports = []
        self.start = None
        self.elems = []
        self.datas = []
        self.data_names = {}
        self.elem_names = {}
        self._collect(sexpr)

    # -- type helpers
    def _type_index(self, params, results):
        key = (tuple(params), tuple(results))
        if key in self.types:
            return self.types.index(key)
        self.types.append(key)
        return len(self.types) - 1

    def _resolve(self, tok, names):
        if isinstance(tok, str) and tok.startswith("$"):
            return names[tok]
        return int(tok)

    def _parse_sig(self, items, f):
        """Consume (type N)? (param ..)* (result ..)* (local ..)*"""
        rest = []
        items = list(items)
        k = 0
        while k < len(items) and isinstance(items[k], list) and items[k] and \
                items[k][0] in ("type", "param", "result", "local"):
            k += 1
        rest = items[k:]
        for it in items[:k]:
            if isinstance(it, list) and it and it[0] == "type":
                f.typeidx = self._resolve(it[1], self.type_names)
            elif isinstance(it, list) and it and it[0] == "param":
                if len(it) >= 2 and it[1].startswith("$"):
                    f.local_names[it[1]] = len(f.params)
                    f.params.append(VALTYPES[it[2]])
                else:
                    f.params += [VALTYPES[t] for t in it[1:]]
            elif isinstance(it, list) and it and it[0] == "result":
                f.results += [VALTYPES[t] for t in it[1:]]
            elif isinstance(it, list) and it and it[0] == "local":
                if len(it) >= 2 and it[1].startswith("$"):
                    f.local_names[it[1]] = len(f.params) + len(f.locals)
                    f.locals.append(VALTYPES[it[2]])
                else:
                    f.locals += [VALTYPES[t] for t in it[1:]]
        return rest

    def _import_other(self, fld, desc):
        """(import "m" "n" (memory $x? min max?)) / (table $x? min max? reftype) /
        (global $x? type | (mut type)): takes the first indices of its kind."""
        imp = (_strbytes(fld[1]), _strbytes(fld[2]))
        rest = desc[1:]
        name = None
        if rest and isinstance(rest[0], str) and rest[0].startswith("$"):
            name, rest = rest[0], rest[1:]
        if desc[0] == "memory":
            if name:
                self.mem_names[name] = len(self.mems)
            nums = [int(x) for x in rest]
            self.mems.append((nums[0], nums[1] if len(nums) > 1 else None, imp))
        elif desc[0] == "table":
            if name:
                self.table_names[name] = len(self.tables)
            nums, rt = [], 0x70
            for it in rest:
                if it in VALTYPES:
                    rt = VALTYPES[it]
                else:
                    nums.append(int(it))
            self.tables.append((rt, nums[0], nums[1] if len(nums) > 1 else None, imp))
        else:
            if name:
                self.global_names[name] = len(self.globals)
            gt = rest[0]
            if isinstance(gt, list) and gt[0] == "mut":
                vt, mut = VALTYPES[gt[1]], 1
            else:
                vt, mut = VALTYPES[gt], 0
            self.globals.append([vt, mut, None, imp])

    def _collect(self, sexpr):
        mod = sexpr[0] if len(sexpr) == 1 and isinstance(sexpr[0], list) else sexpr
        if mod and mod[0] == "module":
            mod = mod[1:]
        if mod and isinstance(mod[0], str) and mod[0].startswith("$"):
            mod = mod[1:]
        # pass 1: types, then imports (indices first), then definitions
        for fld in mod:
            if fld[0] == "type":
                name = fld[1] if isinstance(fld[1], str) else None
                fn = fld[-1]
                f = _Func()
                self._parse_sig(fn[1:], f)
                if name:
                    self.type_names[name] = len(self.types)
                self.types.append((tuple(f.params), tuple(f.results)))
        for fld in mod:
            if fld[0] == "import":
                desc = fld[3]
                if desc[0] in ("memory", "table", "global"):
                    self._import_other(fld, desc)
                    continue
                if desc[0] != "func":
                    raise NotImplementedError("import kind " + desc[0])
                f = _Func()
                f.imported = (_strbytes(fld[1]), _strbytes(fld[2]))
                rest = desc[1:]
                if rest and isinstance(rest[0], str) and rest[0].startswith("$"):
                    f.name = rest[0]
                    rest = rest[1:]
                self._parse_sig(rest, f)
                self._add_func(f)
        defs = []
        for fld in mod:
            k = fld[0]
            if k == "func":
                f = _Func()
                rest = fld[1:]
                if rest and isinstance(rest[0], str) and rest[0].startswith("$"):
                    f.name = rest[0]
                    rest = rest[1:]
                body = []
                for it in rest:
                    if isinstance(it, list) and it and it[0] == "export":
                        f.exports.append(_strbytes(it[1]))
                    else:
                        body.append(it)
                f.body = self._parse_sig(body, f)
                self._add_func(f)
                defs.append(f)
            elif k == "memory":
                rest = fld[1:]
                if rest and isinstance(rest[0], str) and rest[0].startswith("$"):
                    self.mem_names[rest[0]] = len(self.mems)
                    rest = rest[1:]
                nums = []
                for it in rest:
                    if isinstance(it, list) and it[0] == "export":
                        self.exports.append((_strbytes(it[1]), 2, len(self.mems)))
                    else:
                        nums.append(int(it))
                self.mems.append((nums[0], nums[1] if len(nums) > 1 else None))
            elif k == "table":
                rest = fld[1:]
                if rest and isinstance(rest[0], str) and rest[0].startswith("$"):
                    self.table_names[rest[0]] = len(self.tables)
                    rest = rest[1:]
                nums, rt = [], 0x70
                for it in rest:
                    if isinstance(it, list) and it[0] == "export":
                        self.exports.append((_strbytes(it[1]), 1, len(self.tables)))
                    elif it in VALTYPES:
                        rt = VALTYPES[it]
                    else:
                        nums.append(int(it))
                self.tables.append((rt, nums[0], nums[1] if len(nums) > 1 else None))
            elif k == "global":
                rest = fld[1:]
                if rest and isinstance(rest[0], str) and rest[0].startswith("$"):
                    self.global_names[rest[0]] = len(self.globals)
                    rest = rest[1:]
                if isinstance(rest[0], list) and rest[0][0] == "export":
                    self.exports.append((_strbytes(rest[0][1]), 3, len(self.globals)))
                    rest = rest[1:]
                gt = rest[0]
                if isinstance(gt, list) and gt[0] == "mut":
                    vt, mut = VALTYPES[gt[1]], 1
                else:
                    vt, mut = VALTYPES[gt], 0
                self.globals.append([vt, mut, rest[1:]])
            elif k == "export":
                kind = {"func": 0, "table": 1, "memory": 2, "global": 3}[fld[2][0]]
                names = [self.func_names, self.table_names, self.mem_names,
                         self.global_names][kind]
                self.exports.append((_strbytes(fld[1]), kind, fld[2][1]))
                self._pending_names = names
            elif k == "start":
                self.start = fld[1]
            elif k == "elem":
                rest = fld[1:]
                if rest and isinstance(rest[0], str) and rest[0].startswith("$"):
                    self.elem_names[rest[0]] = len(self.elems)
                self.elems.append(rest)
            elif k == "data":
                rest = fld[1:]
                if rest and isinstance(rest[0], str) and rest[0].startswith("$"):
                    self.data_names[rest[0]] = len(self.datas)
                    rest = rest[1:]
                self.datas.append(rest)
        self.defs = defs

    def _add_func(self, f):
        if f.name:
            self.func_names[f.name] = len(self.funcs)
        self.funcs.append(f)

    def _elem_seg(self, rest):
        """One element segment in the binary format's 8 encodings: flags bit 0 passive or
        declarative, bit 1 explicit table index (active) / declarative (passive), bit 2
        items as const expressions."""
        if rest and isinstance(rest[0], str) and rest[0].startswith("$"):
            rest = rest[1:]
        declare = bool(rest) and rest[0] == "declare"
        if declare:
            rest = rest[1:]
        table = None
        if rest and isinstance(rest[0], list) and rest[0][0] == "table":
            table = self._resolve(rest[0][1], self.table_names)
            rest = rest[1:]
        off = None
        if rest and isinstance(rest[0], list) and (rest[0][0] == "offset" or
                                                   rest[0][0].endswith(".const") or
                                                   rest[0][0] == "global.get"):
            off = rest[0][1:] if rest[0][0] == "offset" else [rest[0]]
            rest = rest[1:]
        exprs, rtype = False, 0x70
        if rest and rest[0] in ("funcref", "externref"):
            exprs, rtype = True, VALTYPES[rest[0]]
            rest = rest[1:]
        elif rest and rest[0] == "func":
            rest = rest[1:]
        if exprs:
            items = _vec([self._const_expr([x if x[0] != "item" else x[1]]) for x in rest])
        else:
            items = _vec([uleb(self._resolve(x, self.func_names)) for x in rest])
        if off is not None:
            if table is None:
                return bytes([4 if exprs else 0]) + self._const_expr(off) + items
            return bytes([6 if exprs else 2]) + uleb(table) + self._const_expr(off) + \
                (bytes([rtype]) if exprs else b"\x00") + items
        flags = (3 if declare else 1) | (4 if exprs else 0)
        return bytes([flags]) + (bytes([rtype]) if exprs else b"\x00") + items

    # -- const expressions (globals, offsets)
    def _const_expr(self, items, f=None):
        code = bytearray()
        self._emit_instrs(items, f or _Func(), code, [])
        return bytes(code) + b"\x0b"

    # -- instruction emission
    def _blocktype(self, items, f):
        """Parse optional label + block type at head of items; return (label, bt bytes, rest)."""
        label = None
        i = 0
        if i < len(items) and isinstance(items[i], str) and items[i].startswith("$"):
            label = items[i]
            i += 1
        params, results, tidx = [], [], None
        while i < len(items) and isinstance(items[i], list) and items[i] and \
                items[i][0] in ("param", "result", "type"):
            h = items[i]
            if h[0] == "param":
                params += [VALTYPES[t] for t in h[1:]]
            elif h[0] == "result":
                results += [VALTYPES[t] for t in h[1:]]
            else:
                tidx = self._resolve(h[1], self.type_names)
            i += 1
        if tidx is not None:
            bt = sleb(tidx)
        elif not params and not results:
            bt = b"\x40"
        elif not params and len(results) == 1:
            bt = bytes([results[0]])
        else:
            bt = sleb(self._type_index(params, results))
        return label, bt, items[i:]

    def _label_depth(self, tok, labels):
        if isinstance(tok, str) and tok.startswith("$"):
            for d, l in enumerate(reversed(labels)):
                if l == tok:
                    return d
            raise KeyError(tok)
        return int(tok)

    def _emit_instrs(self, items, f, code, labels):
        """Emit a list of instructions (flat tokens and/or folded lists)."""
        i = 0
        while i < len(items):
            it = items[i]
            if isinstance(it, list):
                self._emit_folded(it, f, code, labels)
                i += 1
                continue
            name = ALIASES.get(it, it)
            if name in ("block", "loop", "if"):
                # flat structured instruction: collect its header
                j = i + 1
                hdr = []
                while j < len(items) and (
                        (isinstance(items[j], str) and items[j].startswith("$") and not hdr)
                        or (isinstance(items[j], list) and items[j] and
                            items[j][0] in ("param", "result", "type"))):
                    hdr.append(items[j])
                    j += 1
                label, bt, _ = self._blocktype(hdr, f)
                code += bytes([OPS[name][0]]) + bt
                labels.append(label)
                i = j
                continue
            if name == "end":
                labels.pop()
                code += b"\x0b"
                i += 1
                if i < len(items) and isinstance(items[i], str) and items[i].startswith("$") \
                        and items[i] not in self.func_names and (
                            i + 1 >= len(items) or True):
                    # optional label after end (only if it was the block's label)
                    pass
                continue
            if name == "else":
                code += b"\x05"
                i += 1
                if i < len(items) and isinstance(items[i], str) and items[i].startswith("$") \
                        and items[i] in labels:
                    i += 1
                continue
            # ordinary instruction with immediates
            n_consumed = self._emit_plain(name, items[i + 1:], f, code, labels)
            i += 1 + n_consumed

    def _emit_folded(self, lst, f, code, labels):
        name = ALIASES.get(lst[0], lst[0])
        if name in ("block", "loop"):
            label, bt, rest = self._blocktype(lst[1:], f)
            code += bytes([OPS[name][0]]) + bt
            labels.append(label)
            self._emit_instrs(rest, f, code, labels)
            labels.pop()
            code += b"\x0b"
            return
        if name == "if":
            label, bt, rest = self._blocktype(lst[1:], f)
            conds = [r for r in rest if not (isinstance(r, list) and r and r[0] in ("then", "else"))]
            thens = [r for r in rest if isinstance(r, list) and r and r[0] == "then"]
            elses = [r for r in rest if isinstance(r, list) and r and r[0] == "else"]
            if not thens and len(conds) >= 2:      # legacy (if cond then-expr else-expr?)
                thens = [["then", conds[1]]]
                if len(conds) > 2:
                    elses = [["else", conds[2]]]
                conds = conds[:1]
            self._emit_instrs(conds, f, code, labels)
            code += b"\x04" + bt
            labels.append(label)
            if thens:
                self._emit_instrs(thens[0][1:], f, code, labels)
            if elses:
                code += b"\x05"
                self._emit_instrs(elses[0][1:], f, code, labels)
            labels.pop()
            code += b"\x0b"
            return
        # plain op: immediates are the leading atoms, operands are nested lists
        atoms = []
        j = 1
        while j < len(lst) and not isinstance(lst[j], list) or \
                (j < len(lst) and isinstance(lst[j], list) and lst[j] and
                 lst[j][0] in ("type", "param", "result") and name in ("call_indirect", "select",
                                                                       "return_call_indirect")):
            atoms.append(lst[j])
            j += 1
        for operand in lst[j:]:
            self._emit_folded(operand, f, code, labels)
        used = self._emit_plain(name, atoms, f, code, labels)
        if used != len(atoms):
            raise SyntaxError("unused immediates in %r" % (lst,))

    def _emit_plain(self, name, toks, f, code, labels):
        """Emit one non-structured instruction; return #tokens consumed from toks."""
        if name not in OPS:
            raise SyntaxError("unknown instruction %r" % name)
        opc, kind, nat_align = OPS[name]
        if opc >= 0xFC00:
            code += bytes([opc >> 8]) + uleb(opc & 0xFF)
        else:
            code.append(opc)
        base_kind = kind & 0xFF
        used = 0

        def tok(k):
            return toks[k] if k < len(toks) else None

        def memref(k, digits=True):   # token k names a memory ($name or index), else None
            t = tok(k)
            if isinstance(t, str) and t in self.mem_names:
                return self.mem_names[t]
            return int(t) if digits and isinstance(t, str) and t.isdigit() else None

        if base_kind == O.NONE:
            pass
        elif base_kind == O.LABEL:
            code += uleb(self._label_depth(toks[0], labels))
            used = 1
        elif base_kind == O.BRTABLE:
            ds = []
            while tok(used) is not None and isinstance(tok(used), str) and \
                    (tok(used).startswith("$") or tok(used).isdigit()):
                ds.append(self._label_depth(tok(used), labels))
                used += 1
            code += uleb(len(ds) - 1) + b"".join(uleb(d) for d in ds)
        elif base_kind == O.FUNC:
            code += uleb(self._resolve(toks[0], self.func_names))
            used = 1
        elif base_kind == O.CALLIND:
            tab = 0
            if tok(0) is not None and not isinstance(tok(0), list):
                tab = self._resolve(toks[0], self.table_names)
                used = 1
            g = _Func()
            sig = []
            while tok(used) is not None and isinstance(tok(used), list):
                sig.append(tok(used))
                used += 1
            self._parse_sig(sig, g)
            ti = g.typeidx if g.typeidx is not None else self._type_index(g.params, g.results)
            code += uleb(ti) + uleb(tab)
        elif base_kind == O.LOCAL:
            t = toks[0]
            code += uleb(f.local_names[t] if t.startswith("$") else int(t))
            used = 1
        elif base_kind == O.GLOBAL:
            code += uleb(self._resolve(toks[0], self.global_names))
            used = 1
        elif base_kind == O.MEM or base_kind == O.MEMLANE:
            off, align = 0, nat_align
            mi = memref(used, base_kind == O.MEM)   # (MultiMemories: the memory before the memarg)
            if mi is not None:
                used += 1
            while tok(used) is not None and isinstance(tok(used), str) and "=" in tok(used):
                k, v = tok(used).split("=")
                if k == "offset":
                    off = int(v, 0)
                elif k == "align":
                    align = int(math.log2(int(v, 0)))
                used += 1
            if mi:   # the reference's memarg order: align | 64, offset, memory index
                code += uleb(align | 64) + uleb(off) + uleb(mi)   # (instruction.cpp:144-156)
            else:
                code += uleb(align) + uleb(off)
            if base_kind == O.MEMLANE:
                code.append(int(toks[used]))
                used += 1
        elif base_kind == O.I32:
            code += sleb(parse_int(toks[0], 32))
            used = 1
        elif base_kind == O.I64:
            code += sleb(parse_int(toks[0], 64))
            used = 1
        elif base_kind == O.F32:
            code += struct.pack("<I", _float_bits(toks[0], 32))
            used = 1
        elif base_kind == O.F64:
            code += struct.pack("<Q", _float_bits(toks[0], 64))
            used = 1
        elif base_kind == O.MEMIDX:
            mi = memref(0)
            code += uleb(mi or 0)
            used = 1 if mi is not None else 0
        elif base_kind == O.MEMMEM:
            a, b = memref(0), memref(1)
            if a is not None and b is not None:
                used = 2
            code += uleb(a or 0) + uleb(b or 0) if used else b"\x00\x00"
        elif base_kind == O.TABLE:
            t = 0
            if tok(0) is not None and isinstance(tok(0), str) and \
                    (tok(0).startswith("$") or tok(0).isdigit()):
                t = self._resolve(tok(0), self.table_names)
                used = 1
            code += uleb(t)
        elif base_kind == O.TWOIDX:
            a = b = 0
            if tok(0) is not None and not isinstance(tok(0), list):
                a = self._resolve(toks[0], self.table_names)
                b = self._resolve(toks[1], self.table_names)
                used = 2
            code += uleb(a) + uleb(b)
        elif base_kind == O.SELECTT:
            if tok(0) is not None and isinstance(tok(0), list) and tok(0)[0] == "result":
                code[-1] = 0x1C
                code += _vec([bytes([VALTYPES[t]]) for t in tok(0)[1:]])
                used = 1
        elif base_kind == O.REFNULL:
            code.append(VALTYPES[{"func": "funcref", "extern": "externref"}.get(toks[0], toks[0])])
            used = 1
        elif base_kind == O.V128:
            shape = toks[0]
            n = {"i8x16": 16, "i16x8": 8, "i32x4": 4, "i64x2": 2, "f32x4": 4, "f64x2": 2}[shape]
            vals = toks[1:1 + n]
            w = 16 // n
            for v in vals:
                if shape.startswith("f"):
                    bits = _float_bits(v, w * 8)
                else:
                    bits = parse_int(v, w * 8) & ((1 << (w * 8)) - 1)
                code += bits.to_bytes(w, "little")
            used = 1 + n
        elif base_kind == O.LANE:
            code.append(int(toks[0]))
            used = 1
        elif base_kind == O.SHUFFLE:
            code += bytes(int(t) for t in toks[:16])
            used = 16
        elif base_kind == O.DATA:
            mi = memref(0) if not kind & 0x100 and tok(1) is not None and not isinstance(tok(1), list) else None
            code += uleb(self._resolve(toks[1 if mi is not None else 0], self.data_names))
            used = 2 if mi is not None else 1
            if not kind & 0x100:
                code += uleb(mi or 0)
        elif base_kind == O.ELEM:
            if kind & 0x100:
                code += uleb(self._resolve(toks[0], self.elem_names))
                used = 1
            else:
                tab = 0
                if len(toks) > 1 and not isinstance(toks[1], list):
                    tab = self._resolve(toks[0], self.table_names)
                    code += uleb(self._resolve(toks[1], self.elem_names)) + uleb(tab)
                    used = 2
                else:
                    code += uleb(self._resolve(toks[0], self.elem_names)) + uleb(0)
                    used = 1
        else:
            raise NotImplementedError(name)
        return used

    # -- final encoding
    def encode(self):
        # resolve function types
        for f in self.funcs:
            if f.typeidx is None:
                f.typeidx = self._type_index(f.params, f.results)
            elif not f.params and not f.results:
                f.params, f.results = list(self.types[f.typeidx][0]), list(self.types[f.typeidx][1])
        for f in self.defs:
            for e in f.exports:
                self.exports.append((e, 0, self.funcs.index(f)))
        bodies = []
        for f in self.defs:
            code = bytearray()
            self._emit_instrs(f.body, f, code, [None])
            code += b"\x0b"
            groups = []
            for t in f.locals:
                if groups and groups[-1][1] == t:
                    groups[-1][0] += 1
                else:
                    groups.append([1, t])
            lb = _vec([uleb(n) + bytes([t]) for n, t in groups])
            body = lb + bytes(code)
            bodies.append(uleb(len(body)) + body)
        globals_enc = []
        for g in self.globals:
            if len(g) == 4:      # imported
                continue
            vt, mut, init = g
            globals_enc.append(bytes([vt, mut]) + self._const_expr(init))
        out = bytearray(b"\x00asm\x01\x00\x00\x00")

        def section(sid, payload):
            out.extend(bytes([sid]) + uleb(len(payload)) + payload)

        if self.types:
            section(1, _vec([b"\x60" + _vec([bytes([p]) for p in ps]) +
                             _vec([bytes([r]) for r in rs]) for ps, rs in self.types]))
        imps = [f for f in self.funcs if f.imported]

        def lim(mn, mx):
            return b"\x00" + uleb(mn) if mx is None else b"\x01" + uleb(mn) + uleb(mx)
        other = []
        for t in self.tables:
            if len(t) == 4:
                other.append(_name(t[3][0]) + _name(t[3][1]) + b"\x01" + bytes([t[0]]) + lim(t[1], t[2]))
        for m in self.mems:
            if len(m) == 3:
                other.append(_name(m[2][0]) + _name(m[2][1]) + b"\x02" + lim(m[0], m[1]))
        for g in self.globals:
            if len(g) == 4:
                other.append(_name(g[3][0]) + _name(g[3][1]) + b"\x03" + bytes([g[0], g[1]]))
        if imps or other:
            section(2, _vec([_name(f.imported[0]) + _name(f.imported[1]) + b"\x00" +
                             uleb(f.typeidx) for f in imps] + other))
        if self.defs:
            section(3, _vec([uleb(f.typeidx) for f in self.defs]))
        tabs = [t for t in self.tables if len(t) == 3]
        if tabs:
            section(4, _vec([bytes([rt]) + lim(mn, mx) for rt, mn, mx in tabs]))
        mems = [m for m in self.mems if len(m) == 2]
        if mems:
            section(5, _vec([lim(mn, mx) for mn, mx in mems]))
        if globals_enc:
            section(6, _vec(globals_enc))
        if self.exports:
            ex = []
            for nm, kind, idx in self.exports:
                names = [self.func_names, self.table_names, self.mem_names, self.global_names][kind]
                ex.append(_name(nm) + bytes([kind]) + uleb(self._resolve(idx, names)
                                                           if not isinstance(idx, int) else idx))
            section(7, _vec(ex))
        if self.start is not None:
            section(8, uleb(self._resolve(self.start, self.func_names)))
        if self.elems:
            segs = []
            for e in self.elems:
                segs.append(self._elem_seg(list(e)))
            section(9, _vec(segs))
        if self.datas and any(1 for d in self.datas):
            pass
        if bodies:
            section(10, _vec(bodies))
        if self.datas:
            segs = []
            for d in self.datas:
                rest = list(d)
                mi = 0
                if rest and isinstance(rest[0], list) and rest[0][0] == "memory":
                    mi = self._resolve(rest[0][1], self.mem_names)
                    rest = rest[1:]
                if rest and isinstance(rest[0], list):
                    off = rest[0]
                    if off[0] == "offset":
                        off = off[1:]
                    else:
                        off = [off]
                    data = b"".join(_strbytes(s) for s in rest[1:])
                    head = b"\x02" + uleb(mi) if mi else b"\x00"   # (segment.cpp:316-323)
                    segs.append(head + self._const_expr(off) + uleb(len(data)) + data)
                else:
                    data = b"".join(_strbytes(s) for s in rest)
                    segs.append(b"\x01" + uleb(len(data)) + data)
            section(11, _vec(segs))
        return bytes(out)


def assemble(src):
    """Assemble WAT source text into a wasm binary (bytes)."""
    return Assembler(_parse(_tokenize(src))).encode()
