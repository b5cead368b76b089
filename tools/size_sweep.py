"""Headline C2 pipeline at several batch sizes (per-item stage times), to see
the grid-tail effect: a launch of 1M lanes is 15,628 waves against 3,072
resident-wave slots (1,024 SIMDs x 3 waves), i.e. 5.09 rounds.
usage: size_sweep.py n1,n2,..."""
import json
import subprocess
import sys

for n in [int(x) for x in sys.argv[1].split(",")]:
    r = subprocess.run([sys.executable, "bench.py", "--n", str(n), "--steps", "5", "--warmup", "2", "--no-extras",
                        "--no-latency", "--no-cpu-baseline"], capture_output=True, text=True, timeout=300)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    p = d["pipeline"]
    print(json.dumps({"n": n, "Mverifies_s": round(d["value"] / 1e6, 2),
                      "us_per_1k_items": {k: round(v / n * 1e6, 3) for k, v in p.items() if k.endswith("_ms")}}),
          flush=True)
