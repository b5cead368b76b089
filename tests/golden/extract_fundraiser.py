"""Extract the fundraiser known-answer vectors (priv, pub, addr) from the
reference's crypto/hd/testdata/test.json (data read by
crypto/hd/fundraiser_test.go:49-88) into tests/golden/fundraiser_kat.json.
Run in the build container (the GPU box has no /root/reference):
    python tests/golden/extract_fundraiser.py /root/reference/crypto/hd/testdata/test.json
"""
import json
import os
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/crypto/hd/testdata/test.json"
rows = json.load(open(src))
out = {"source": "crypto/hd/testdata/test.json (all %d entries; priv/pub/addr fields) -- reference known-answer "
                 "data used by crypto/hd/fundraiser_test.go:49-88" % len(rows),
       "vectors": [{"priv": r["priv"], "pub": r["pub"], "addr": r["addr"]} for r in rows]}
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fundraiser_kat.json")
with open(dst, "w") as f:
    json.dump(out, f, indent=0)
print(len(rows), "vectors ->", dst)
