"""Static path length of one converged dispatch in the interpreter kernel's ISA.

usage: python tools/isa_path.py <kernel.s> <op number> [op number ...]

Walks the gfx950 assembly of wb_exec_kernel from the dispatch-loop header, evaluating the
scalar compare tree on the opcode register (and SGPR boolean flow masks set on the way)
for the given opcode, and counts instructions by class until control returns to the
loop header. Branches on unknown values (per-lane data, trap checks) take the
fall-through and are reported. A tuning aid for the dispatch overhead; not a test.
"""
import re
import sys
TRACE = False


def parse(path):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith("wb_exec_kernel:"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    ins, labels = [], {}
    for l in lines[start:end]:
        s = l.split(";")[0].strip()
        if not s or s.startswith("."):
            m = re.match(r"^(\.LBB\d+_\d+):", l)
            if m:
                labels[m.group(1)] = len(ins)
            continue
        if s.endswith(":"):
            continue
        ins.append(s)
    return ins, labels


def header(lines_path):
    """Loop header = the block annotated 'This Loop Header: Depth=2' (the run loop)."""
    txt = open(lines_path).read().splitlines()
    for i, l in enumerate(txt):
        if "This Loop Header: Depth=2" in l:
            for j in range(i, 0, -1):
                m = re.match(r"^(\.LBB\d+_\d+):", txt[j])
                if m:
                    return m.group(1)
    raise SystemExit("no depth-2 loop header")


def reg64(r):
    m = re.match(r"s\[(\d+):(\d+)\]", r)
    return ("s", int(m.group(1))) if m else (r,)


# Outcomes assumed for compares on values the tracer cannot know, chosen to follow the
# steady converged path: tick countdown not expired, all lanes agree on the next pc, no
# lane left the run, the next pc is the fall-through.
ASSUME = {("lg", "0"): True, ("lg", "u64"): False, ("ge", "u32"): False, ("eq", "u32"): True}


def run(path, op, ctl=False):
    ins, labels = parse(path)
    h = labels[header(path)]
    # the opcode register: first s_sext_i32_i16 / s_and_b32 ..., 0xffff after the header
    opreg = w0reg = None
    for k in range(h, h + 40):
        m = re.match(r"s_sext_i32_i16 (s\d+), (s\d+)", ins[k])
        if m and opreg is None:
            opreg, w0reg = m.group(1), m.group(2)
    regs = {opreg: op}
    scc, counts, unknown = None, {}, []
    execops = []
    pc, steps = h, 0
    while steps < 4000:
        steps += 1
        s = ins[pc]
        if TRACE: print("   ", s)
        mnem = s.split()[0]
        cls = ("branch" if mnem.startswith("s_cbranch") or mnem == "s_branch" else
               "salu" if mnem.startswith("s_") else "valu" if mnem.startswith("v_") else
               "lds" if mnem.startswith("ds_") else "vmem" if mnem.startswith(("global_", "buffer_")) else
               "other")
        if mnem != "s_waitcnt" and not s.startswith(";"):
            counts[cls] = counts.get(cls, 0) + 1
        if mnem == "s_waitcnt":
            counts["waitcnt"] = counts.get("waitcnt", 0) + 1
        if "saveexec" in mnem or mnem.startswith("s_cbranch_exec") or \
                (mnem.endswith("_b64") and s.split()[1].rstrip(",") == "exec"):
            execops.append(s)
        args = [a.strip() for a in s[len(mnem):].split(",")]
        val = lambda a: (int(a, 0) if re.match(r"^-?(0x)?[0-9a-fA-F]+$", a) else regs.get(a))
        if mnem.startswith(("s_cmpk_", "s_cmp_")):
            kind = mnem.split("_")[2]
            x, y = val(args[0]), val(args[1])
            if args[0] == w0reg and args[1] == "-1" and kind == "gt":
                scc = not ctl                       # CTL bit (w0 bit 31) clear?
            elif x is None or y is None:
                key = (kind, "0" if args[1] == "0" else mnem.split("_")[-1])
                scc = ASSUME.get(key)
            else:
                scc = {"lt": x < y, "gt": x > y, "eq": x == y, "lg": x != y, "le": x <= y,
                       "ge": x >= y}.get(kind)
        elif mnem == "s_mov_b64" and args[1] in ("-1", "0"):
            regs[reg64(args[0])] = args[1] == "-1"
        elif mnem == "s_cselect_b64" and args[1] == "-1" and args[2] == "0":
            regs[reg64(args[0])] = scc
        elif mnem in ("s_and_b64", "s_or_b64", "s_andn2_b64"):
            a = True if args[1] == "exec" else regs.get(reg64(args[1]))
            b = True if args[2] == "exec" else regs.get(reg64(args[2]))
            r = None
            if a is not None and b is not None:
                r = a and b if mnem == "s_and_b64" else a or b if mnem == "s_or_b64" else a and not b
            if args[0] == "vcc":
                regs["vcc"] = r
            elif args[0] != "exec":
                regs[reg64(args[0])] = r
        elif mnem.startswith("s_cbranch"):
            c = mnem[len("s_cbranch_"):]
            t = {"scc1": scc, "scc0": None if scc is None else not scc,
                 "vccz": None if regs.get("vcc") is None else not regs["vcc"],
                 "vccnz": regs.get("vcc"), "execz": False, "execnz": True}[c]
            if t is None:
                unknown.append((pc, s))
                t = False
            if t:
                pc = labels[args[0]]
                if pc == h:
                    break
                continue
        elif mnem == "s_branch":
            pc = labels[args[0]]
            if pc == h:
                break
            continue
        elif mnem == "s_sext_i32_i16" and args[0] == opreg:
            regs[opreg] = op
        elif mnem.startswith(("s_", "v_")) and args and re.match(r"^s\d+$", args[0]):
            regs.pop(args[0], None)
        pc += 1
        if pc == h:
            break
    counts["exec"] = len(execops)
    return counts, unknown, steps


def names():
    import os
    src = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "wasmedge_amd",
                            "csrc", "dbc.h")).read()
    i = src.index("#define DBC_OPS(X)")
    return re.findall(r"X\((\w+)\)", src[i:src.index("\n\n", i)])


if __name__ == "__main__" and sys.argv[2:] == ["--divergent"]:
    for k, nm in enumerate(names()):
        c, unk, n = run(sys.argv[1], k)
        if c.get("exec"):
            print("%3d %-22s exec-ops %d  total %d" % (k, nm, c["exec"], sum(
                v for kk, v in c.items() if kk not in ("waitcnt", "exec"))))
    sys.exit(0)

if __name__ == "__main__":
    for o in sys.argv[2:]:
        ctl = o.endswith("c")                   # e.g. 19c: the instruction has CTL set
        c, unk, n = run(sys.argv[1], int(o.rstrip("c"), 0), ctl)
        tot = sum(v for k, v in c.items() if k != "waitcnt")
        print("op %-5s total %3d  %s  unknown-branches %d" % (o, tot, c, len(unk)))
        for u in unk[:6]:
            print("    ?", u[1])
