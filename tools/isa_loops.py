"""Loops of one kernel in a gfx950 assembly file (no GPU): every backward branch target .. branch range, with its
static instruction mix by class (mfma / valu / trans / salu / vmem / ds / wait / scratch), for the per-iteration
budget of a hot loop. usage: python tools/isa_loops.py file.s kernel_symbol"""
import collections
import re
import sys


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_rcp", "v_log", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "trans"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("ds_"):
        return "ds"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return None


def main(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    instrs = []   # (line index, op, text)
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = len(instrs)
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        instrs.append((i, op, t))
    loops = []
    for k, (i, op, t) in enumerate(instrs):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = t.split()[-1]
            if tgt in labels and labels[tgt] <= k:
                loops.append((labels[tgt], k))
    for a, b in sorted(loops, key=lambda x: x[0] - x[1]):
        mix = collections.Counter(classify(op) for _, op, _ in instrs[a:b + 1])
        mix.pop(None, None)
        if b - a < 30:
            continue
        ops = collections.Counter(op for _, op, _ in instrs[a:b + 1] if classify(op) == "valu")
        print(f"loop instrs [{a}, {b}] ({b - a + 1}): {dict(mix)}")
        print("   top valu:", ops.most_common(18))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
