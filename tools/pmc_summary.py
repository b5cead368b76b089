"""Summarise a tools/pmc_round.sh run into one JSON per kernel (per launch).

FETCH_SIZE / WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md (HBM section),
FETCH_SIZE on gfx950 reports half the bytes of a wide coalesced read, so the
corrected fetch is 2x the counter; WRITE_SIZE is taken as-is.  SQ counters:
SQ_INSTS_VALU is per-wave instructions (one lane of the verify = one wave slot),
SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / SQ_ACTIVE_* count quad-cycles, GRBM_GUI_ACTIVE
is summed over the 8 XCDs.

usage: pmc_summary.py <run_dir> <items_per_launch> <out.json>
"""
import collections
import csv
import json
import os
import sys


def load(d, name):
    p = os.path.join(d, name, "run_counter_collection.csv")
    if not os.path.exists(p):
        return {}
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(p)):
        # "void gv::k_ecmult<false>(...)" -> "k_ecmult" (the bench runs one instance of each)
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("gv::", "").strip()
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def main():
    d, n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    merged = collections.defaultdict(dict)
    for p in ("fetch", "write", "sq1", "sq2"):
        for k, cs in load(d, p).items():
            merged[k].update(cs)
    res = {"items_per_launch": n, "source": d, "kernels": {}}
    for k, c in merged.items():
        e = {"counters": c}
        if "FETCH_SIZE" in c:
            e["fetch_bytes_corrected"] = c["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in c:
            e["write_bytes"] = c["WRITE_SIZE"] * 1024
        if "fetch_bytes_corrected" in e and "write_bytes" in e:
            e["hbm_bytes"] = e["fetch_bytes_corrected"] + e["write_bytes"]
            e["hbm_bytes_per_item"] = e["hbm_bytes"] / n
        if "SQ_INSTS_VALU" in c and k != "k_gen_gtable":
            e["valu_insts_per_item"] = c["SQ_INSTS_VALU"] / (n / 64.0) if k != "k_scalar_inv" else c["SQ_INSTS_VALU"] / (n / 64.0)
        if "GRBM_GUI_ACTIVE" in c and "SQ_ACTIVE_INST_VALU" in c:
            simd_cycles = c["GRBM_GUI_ACTIVE"] / 8.0 * 1024          # 256 CUs x 4 SIMDs
            e["valu_busy_frac"] = c["SQ_ACTIVE_INST_VALU"] * 4 / simd_cycles
        res["kernels"][k] = e
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, e in res["kernels"].items():
        print(k, {x: (round(v, 3) if isinstance(v, float) else v) for x, v in e.items() if x != "counters"})


if __name__ == "__main__":
    main()
