"""GPU tests of the account pubkey cache (gv_keys_load + keyed verifies,
SURVEY.md §8f-2): a keyed verify must give exactly the verdict of the pub33
path -- hence of the oracle -- for the key loaded into the slot, including keys
ParsePubKey rejects and slots that were never loaded."""
import numpy as np
import pytest

import gpuverify as gvm
from golden_io import load_digest_vectors, load_msg_vectors
from oracle import oracle as O
from test_gpu_parity import PATHS, make_random_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ver():
    v = gvm.Verifier([0])
    yield v
    v.close()


# (lat_max, sliced, keys_k6, keys_wide, lat_kw): the PATHS schedules (rows: pub33
# only) with the resident arena's wide-window tables (small batches:
# k_verify_lat16_kw), plus the sliced kernel on the kn tables (lat_kw 0) and on
# the k4 tables, and the throughput ladders on the k6 tables and the two-window layout
KEYED_PATHS = {**{p: (v[0], v[1], 1, 2, 1) for p, v in PATHS.items() if p != "latency_rows"},
               "latency_kn_arena": (1 << 30, 1, 1, 2, 0),
               "latency_k4_arena": (1 << 30, 1, 0, 0, 1), "throughput_k6_arena": (0, 1, 1, 0, 1),
               "throughput_wide_two": (0, 1, 1, 1, 1)}


@pytest.fixture(params=sorted(KEYED_PATHS))
def path(request, ver):
    """Keyed batches take the fused small-batch kernel up to lat_max
    (k_verify_lat16_kw on the arena's one-window wide tables,
    k_verify_lat16_kn on its kn tables with lat_kw 0, k_verify_lat16_sl on its
    k4 tables with keys_k6 0, or k_verify_lat16 with lat_sliced 0), the
    throughput pipeline above it: every schedule is checked."""
    lat_max, sliced, keys_k6, keys_wide, lat_kw = KEYED_PATHS[request.param]
    ver.set_option("lat_kw", lat_kw)
    ver.set_option("lat_max", lat_max)
    ver.set_option("lat_sliced", sliced)
    ver.set_option("lat_sl_max", 1 << 30)
    ver.set_option("keys_k6", keys_k6)
    ver.set_option("keys_wide", keys_wide)
    yield request.param
    ver.reset_schedule()
    ver.set_option("lat_sliced", 1)
    ver.set_option("keys_k6", 1)
    ver.set_option("keys_wide", 2)
    ver.set_option("lat_kw", 1)


def keyed_inputs(ver, pub):
    """Load the distinct keys of `pub` (in first-seen order) and map items to slots."""
    uniq, first, inv = np.unique(pub, axis=0, return_index=True, return_inverse=True)
    order = np.argsort(first)
    slots = ver.keys_load(uniq[order])
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    return slots[rank[inv.reshape(-1)]]


def test_golden_vectors_keyed(ver, path):
    ver.keys_reset()
    pub, sig, dig, ok, cats = load_digest_vectors()
    got = ver.verify_batch_digests_keyed(keyed_inputs(ver, pub), sig, dig)
    bad = [(i, cats[i], int(ok[i])) for i in range(len(ok)) if got[i] != ok[i]]
    assert not bad, bad[:20]
    pub, sig, msgs, ok, cats = load_msg_vectors()
    got = ver.verify_batch_msgs_keyed(keyed_inputs(ver, pub), sig, msgs)
    bad = [(i, cats[i], int(ok[i])) for i in range(len(ok)) if got[i] != ok[i]]
    assert not bad, bad[:20]


def test_adversarial_keyed_equals_oracle_and_pub_path(ver, path):
    ver.keys_reset()
    pub, sig, dig = make_random_batch(20000, seed=0xCA, adversarial=0.25, nkeys=301)
    want = O.verify_digests(pub, sig, dig, threads=16)
    slots = keyed_inputs(ver, pub)
    got = ver.verify_batch_digests_keyed(slots, sig, dig)
    assert np.array_equal(got, want)
    assert np.array_equal(got, ver.verify_batch_digests(pub, sig, dig))


@pytest.mark.parametrize("n", [1, 17, 255, 256, 257, 3000])
def test_ragged_keyed_and_unloaded_slots(ver, n, path):
    ver.keys_reset()
    pub, sig, dig = make_random_batch(n, seed=1000 + n, adversarial=0.3, nkeys=5)
    want = O.verify_digests(pub, sig, dig, threads=8)
    slots = keyed_inputs(ver, pub)
    assert np.array_equal(ver.verify_batch_digests_keyed(slots, sig, dig), want)
    # a slot that was never loaded is false, whatever the signature
    bad = slots.copy()
    bad[::3] = ver.keys_count + np.arange(len(bad[::3]), dtype=np.uint32)
    exp = want.copy()
    exp[::3] = 0
    assert np.array_equal(ver.verify_batch_digests_keyed(bad, sig, dig), exp)


def test_arena_growth_keeps_earlier_slots(ver):
    """Many loads grow the arena (re-allocation + copy); earlier slots stay valid."""
    ver.keys_reset()
    pub, sig, dig = make_random_batch(6000, seed=31, adversarial=0.2, nkeys=6000)
    want = O.verify_digests(pub, sig, dig, threads=16)
    slots = np.concatenate([ver.keys_load(pub[i:i + 1500]) for i in range(0, 6000, 1500)])
    assert ver.keys_count == 6000 and np.array_equal(slots, np.arange(6000))
    assert np.array_equal(ver.verify_batch_digests_keyed(slots, sig, dig), want)


def test_device_resident_keyed(ver):
    ver.keys_reset()
    n = 5000
    pub, sig, dig = make_random_batch(n, seed=41, adversarial=0.25, nkeys=97)
    want = O.verify_digests(pub, sig, dig, threads=16)
    slots = keyed_inputs(ver, pub)
    bufs = [ver.dev_alloc(a.nbytes) for a in (slots, sig, dig)]
    d_bits = ver.dev_alloc(((n + 63) // 64) * 8)
    try:
        for p, a in zip(bufs, (slots, sig, dig)):
            ver.dev_upload(p, a)
        ver.dev_verify_digests_keyed(0, n, bufs[0], bufs[1], bufs[2], d_bits)
        bits = np.zeros((n + 63) // 64, dtype=np.uint64)
        ver.dev_download(bits, d_bits)
    finally:
        for p in bufs + [d_bits]:
            ver.dev_free(p)
    got = np.unpackbits(bits.view(np.uint8), bitorder="little")[:n]
    assert np.array_equal(got, want)


def test_keyed_two_device_slots():
    pub, sig, dig = make_random_batch(3001, seed=78, adversarial=0.25, nkeys=13)
    want = O.verify_digests(pub, sig, dig, threads=16)
    with gvm.Verifier([0, 0]) as v2:
        slots = keyed_inputs(v2, pub)
        assert np.array_equal(v2.verify_batch_digests_keyed(slots, sig, dig), want)
