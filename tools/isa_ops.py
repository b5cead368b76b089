"""Per-operation gfx950 instruction counts of the k_ecmult_k4 ladder.

Compiles tools/isa_ops.hip (one straight-line kernel per ladder operation,
built from the product sources with the exceptional branches compiled out) to
device assembly and counts each kernel's instructions by class, minus the
load/store frame.  Then weights the counts by the ladder's operation counts
per verify (derived from the ladder's schedule in gv_kernels.hip k_ecmult_k4:
6 x 5 doublings, 52 Q adds of which 26 lambda-Q, 11 G adds, one final check;
--glv: the 14 G adds of the GLV G schedule)
and prints the predicted VALU instructions per verify next to the PMC figure.

Usage: python tools/isa_ops.py [--json out.json] [--defs "-DFOO=1"]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "isa_ops.hip")

# operations per verify of k_ecmult_k4<true> (schedule: positions 6..0, 5
# doublings between positions; Q windows per group 7, 7, 6, 6 -> 26 per GLV
# half, each with a Q and a lambda-Q digit -- the lambda-Q entries added as
# plain Q additions on lambda^2 (acc), entered and left by a beta product at
# each of the 7 positions (GV_LAMFRAME); G: 11 25-bit windows of the unsplit u1)
LADDER_OPS = {"isa_dbl": 30, "isa_addq": 52, "isa_mul": 14, "isa_addg": 11, "isa_finish": 1}
# without the lambda frame (GV_LAMFRAME=0): a beta product inside each lambda-Q addition
LADDER_OPS_NOFRAME = {"isa_dbl": 30, "isa_addq": 26, "isa_addlq": 26, "isa_addg": 11, "isa_finish": 1}
# the GLV G schedule (gv_set_option "gfull" 0): 7 20-bit windows per GLV half
LADDER_OPS_GLV = dict(LADDER_OPS, isa_addg=14)


def classify(op):
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("v_mad_u64_u32"):
        return "mad64"
    if op.startswith(("v_mul_lo", "v_mul_hi", "v_mad_u32")):
        return "mul32"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer")):
        return "smem"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def kernels(asm):
    out = {}
    for m in re.finditer(r"^(_ZN2gv(\d+)(isa_\w+?)E\w*):", asm, re.M):
        name = m.group(3)
        body = asm[m.end():]
        body = body[:body.index(".Lfunc_end")]
        ops = []
        for line in body.split("\n"):
            s = line.strip()
            if not s or s.startswith((".", ";", "//")) or s.endswith(":"):
                continue
            ops.append(s.split()[0])
        by_class = collections.Counter(classify(o) for o in ops)
        by_op = collections.Counter(ops)
        vgpr = re.search(r"\.set " + re.escape(m.group(1)) + r"\.num_vgpr, (\d+)", asm)
        out[name] = {"total": len(ops), "class": dict(by_class), "top": dict(by_op.most_common(12)),
                     "vgpr": int(vgpr.group(1)) if vgpr else None}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    ap.add_argument("--defs", default="")
    ap.add_argument("--asm", default="/tmp/isa_ops.s")
    ap.add_argument("--glv", action="store_true", help="the GLV G schedule (14 G additions)")
    a = ap.parse_args()
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
           SRC, "-o", a.asm] + a.defs.split()
    subprocess.run(cmd, check=True, cwd=os.path.join(ROOT, "cosmos-sdk-rootchain_amd"))
    k = kernels(open(a.asm).read())
    frame = k["isa_frame"]["class"]
    rows = {}
    for name, v in sorted(k.items()):
        if name == "isa_frame":
            continue
        net = dict(v["class"])
        if name != "isa_finish":
            for c, n in frame.items():
                net[c] = net.get(c, 0) - n
        v["net"] = net
        rows[name] = v
        valu = net.get("mad64", 0) + net.get("mul32", 0) + net.get("valu", 0)
        print(f"{name:11s} mad64 {net.get('mad64', 0):5d}  other VALU {net.get('mul32', 0) + net.get('valu', 0):5d}"
              f"  VALU {valu:5d}  s_nop {net.get('s_nop', 0):4d}  vmem {net.get('vmem', 0):3d}")
    ops = LADDER_OPS_GLV if a.glv else LADDER_OPS
    pred = collections.Counter()
    for name, cnt in ops.items():
        for c, n in rows[name]["net"].items():
            pred[c] += cnt * n
    valu = pred["mad64"] + pred["mul32"] + pred["valu"]
    print(f"per verify (ops {ops}): mad64 {pred['mad64']}, other VALU {pred['mul32'] + pred['valu']}, "
          f"VALU {valu}, s_nop {pred['s_nop']}")
    if a.json:
        json.dump({"ladder_ops_per_verify": ops, "per_op": rows, "per_verify": dict(pred),
                   "valu_per_verify": valu, "defs": a.defs}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    sys.exit(main())
