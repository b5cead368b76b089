"""Print the C1 / C4 / message-path lines of a bench.py JSON (stdin or file)."""
import json
import sys

d = json.loads((open(sys.argv[1]) if len(sys.argv) > 1 else sys.stdin).read().strip().splitlines()[-1])
ex = d.get("extras", {})
c1 = ex.get("c1_ante", {})
print(json.dumps({"value": d["value"], "c1_steady": c1.get("block_path_steady"), "c1_first": c1.get("block_path"),
                  "checktx_window": c1.get("checktx_window", {}).get("txs_per_s"),
                  "c4": {k: ex.get("c4_multisig", {}).get(k) for k in ("leaves_per_s", "gpu_s", "preverify_s", "seconds")}}))
