"""Key-ordered lanes (gv_set_option "sort_keys", csrc/gv_sort.hip): keyed
throughput batches on the 4-group ladder sort their lanes by key slot, read the
signature / digest (or message) of item perm[lane], and gather the accept
bits back to item order.  The verdicts must be exactly the item-order ones --
for grouped keys (repeated rejected keys included), cached slots with
never-loaded slots interleaved, ragged sizes and the message path."""
import numpy as np
import pytest

import bench
import gpuverify as gvm
from golden_io import load_digest_vectors, load_msg_vectors
from oracle import oracle as O
from test_gpu_parity import make_random_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ver():
    v = gvm.Verifier([0])
    yield v
    v.set_option("sort_keys", 1)
    v.close()


def both(ver, fn):
    ver.set_option("sort_keys", 1)
    a = fn()
    ver.set_option("sort_keys", 0)
    b = fn()
    ver.set_option("sort_keys", 1)
    return a, b


@pytest.mark.parametrize("n", [16_384, 16_447, 70_001])
def test_grouped_route_sorted_equals_item_order(ver, n):
    pub, sig, dig, exp = bench.make_digest_workload(n, 0x70 + n % 7, 1000, 0.25, 16)
    g0, _ = ver.group_stats()
    a, b = both(ver, lambda: ver.verify_batch_digests(pub, sig, dig))
    assert ver.group_stats()[0] - g0 == 2
    assert np.array_equal(a, exp) and np.array_equal(b, exp)


def test_grouped_goldens_tiled_sorted(ver):
    """every rejection class (bad prefixes, x >= p, non-residues, infinity,
    x in [n, p)) tiled and shuffled: rejected keys sort into their own slots"""
    gp, gs, gd, gok, _ = load_digest_vectors()
    reps = 120
    perm = np.random.default_rng(11).permutation(reps * len(gp))
    pub, sig, dig = (np.tile(x, (reps, 1))[perm] for x in (gp, gs, gd))
    exp = np.tile(gok, reps)[perm]
    a, b = both(ver, lambda: ver.verify_batch_digests(pub, sig, dig))
    assert np.array_equal(a, exp) and np.array_equal(b, exp)
    d = [ver.dev_alloc(x.nbytes) for x in (pub, sig, dig)]
    n = len(exp)
    d_bits = ver.dev_alloc(((n + 63) // 64) * 8)
    try:
        for p, x in zip(d, (pub, sig, dig)):
            ver.dev_upload(p, x)
        for _ in range(2):                          # pipelined consecutive calls
            ver.dev_verify_digests(0, n, d[0], d[1], d[2], d_bits)
        ver.dev_sync()
        bits = np.zeros((n + 63) // 64, np.uint64)
        ver.dev_download(bits, d_bits)
    finally:
        for p in d + [d_bits]:
            ver.dev_free(p)
    assert np.array_equal(bench.unpack_bits(bits, n), exp)


def test_cached_slots_with_unloaded_slots_sorted(ver):
    ver.keys_reset()
    n = 40_000
    pub, sig, dig = make_random_batch(n, seed=0x5A, adversarial=0.25, nkeys=257)
    want = O.verify_digests(pub, sig, dig, threads=16)
    uniq, inv = np.unique(pub, axis=0, return_inverse=True)
    slots = ver.keys_load(uniq)[inv.reshape(-1)].astype(np.uint32)
    bad = slots.copy()
    bad[::5] = ver.keys_count + np.arange(len(bad[::5]), dtype=np.uint32)   # never loaded: false
    exp = want.copy()
    exp[::5] = 0
    a, b = both(ver, lambda: ver.verify_batch_digests_keyed(slots, sig, dig))
    assert np.array_equal(a, want) and np.array_equal(b, want)
    a, b = both(ver, lambda: ver.verify_batch_digests_keyed(bad, sig, dig))
    assert np.array_equal(a, exp) and np.array_equal(b, exp)


def test_message_path_sorted(ver):
    mp, ms, mm, mok, _ = load_msg_vectors()
    reps = max(1, 40_000 // len(mp))
    perm = np.random.default_rng(12).permutation(reps * len(mp))
    pub, sig = np.tile(mp, (reps, 1))[perm], np.tile(ms, (reps, 1))[perm]
    msgs = [(mm * reps)[i] for i in perm]
    exp = np.tile(mok, reps)[perm]
    a, b = both(ver, lambda: ver.verify_batch_msgs(pub, sig, msgs))
    assert np.array_equal(a, exp) and np.array_equal(b, exp)
    ver.keys_reset()
    uniq, inv = np.unique(pub, axis=0, return_inverse=True)
    slots = ver.keys_load(uniq)[inv.reshape(-1)].astype(np.uint32)
    a, b = both(ver, lambda: ver.verify_batch_msgs_keyed(slots, sig, msgs))
    assert np.array_equal(a, exp) and np.array_equal(b, exp)
