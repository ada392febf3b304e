"""Static instruction mix of the gfx950 kernels in one HIP source (no GPU needed).

usage: python tools/isa_mix.py [csrc/agent_fwd.hip] [kernel-substring]
Compiles the device code to assembly with hipcc and prints, per kernel symbol,
counts by class (mfma / valu / salu / vmem / ds / scratch) plus VGPR/SGPR/spill
metadata and the most frequent VALU opcodes.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mini-marl_amd")


def assemble(src):
    out = os.path.join(tempfile.mkdtemp(), "k.s")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                           "--cuda-device-only", "-S", "-I" + os.path.join(ROOT, "include"),
                           "-I" + os.path.join(PKG, "csrc"), src, "-o", out])
    return open(out).read()


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
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


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(PKG, "csrc", "agent_fwd.hip")
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    asm = assemble(src)
    cur, kern = None, {}
    meta = {}
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            kern[cur] = collections.Counter()
            continue
        if line.startswith("\t.end_amdhsa_kernel") or line.startswith(".Lfunc_end"):
            cur = None
        for key in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "agpr_count"):
            m = re.match(r"\s*\.%s:\s+(\d+)" % key, line)
            if m:
                meta.setdefault(key, []).append(int(m.group(1)))
        if cur is None:
            continue
        t = line.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        kern[cur][t[0]] += 1
    names = [k for k in kern if filt in k and sum(kern[k].values())]
    for k in names:
        c = kern[k]
        cls = collections.Counter()
        for op, n in c.items():
            x = classify(op)
            if x:
                cls[x] += n
        print(k[:110])
        print("  ", dict(cls.most_common()))
        print("   top valu:", [(op, n) for op, n in c.most_common() if classify(op) == "valu"][:14])
    print("metadata (all kernels, in order):", {k: v for k, v in meta.items()})


if __name__ == "__main__":
    main()
