"""C2 keyed line alone (tools/bench_extras.c2_key_cache) on the bench workload,
for A/B runs of the keyed ladder (GV_KEYED_K4=0/1).  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tools import bench_extras  # noqa: E402


def main():
    n = int(os.environ.get("GV_PROBE_N", "1000000"))
    pub, sig, dig, exp = bench.make_digest_workload(n, 0xC2, 65536, 0.0, 16)
    ver = bench.gvm.Verifier([0])
    out = bench_extras.c2_key_cache(ver, pub, sig, dig, exp, 65536, steps=5)
    out["keyed_k4"] = os.environ.get("GV_KEYED_K4", "1")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
