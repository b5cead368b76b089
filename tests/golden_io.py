"""Load the committed golden fixtures as numpy batches (test helper)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_digest_vectors():
    vs = json.load(open(os.path.join(GOLDEN, "vectors_digest.json")))
    pub = np.array([np.frombuffer(bytes.fromhex(v["pub"]), np.uint8) for v in vs])
    sig = np.array([np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vs])
    dig = np.array([np.frombuffer(bytes.fromhex(v["dig"]), np.uint8) for v in vs])
    ok = np.array([v["ok"] for v in vs], dtype=np.uint8)
    cats = [v["cat"] for v in vs]
    return pub, sig, dig, ok, cats


def load_msg_vectors():
    vs = json.load(open(os.path.join(GOLDEN, "vectors_msg.json")))
    pub = np.array([np.frombuffer(bytes.fromhex(v["pub"]), np.uint8) for v in vs])
    sig = np.array([np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vs])
    msgs = [bytes.fromhex(v["msg"]) for v in vs]
    ok = np.array([v["ok"] for v in vs], dtype=np.uint8)
    cats = [v["cat"] for v in vs]
    return pub, sig, msgs, ok, cats
