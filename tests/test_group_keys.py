"""In-batch key grouping (gv_set_option "group_keys"): a pub33 batch whose
items repeat keys parses each distinct key once (k_dedupe*, k_keys_chain + k_keys_tables into a
per-batch arena) and runs the keyed pipeline.  The verdicts must be exactly the
per-item pub33 pipeline's -- including keys that ParsePubKey rejects (repeated
bad prefixes, x >= p, non-residue x), which get a slot too and make every item
on them false -- and the route is taken only below the distinct-key bound."""
import numpy as np
import pytest

import bench
import gpuverify as gvm
from golden_io import load_digest_vectors
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ver():
    v = gvm.Verifier([0])
    yield v
    v.close()


def grouped_vs_plain(ver, pub, sig, dig, msgs=None):
    b0, _ = ver.group_stats()
    ver.set_option("group_keys", 1)
    got = ver.verify_batch_digests(pub, sig, dig) if msgs is None else ver.verify_batch_msgs(pub, sig, msgs)
    b1, k1 = ver.group_stats()
    ver.set_option("group_keys", 0)
    ref = ver.verify_batch_digests(pub, sig, dig) if msgs is None else ver.verify_batch_msgs(pub, sig, msgs)
    ver.set_option("group_keys", 1)
    return got, ref, b1 - b0


def test_repeated_keys_take_the_grouped_route_with_identical_verdicts(ver):
    pub, sig, dig, exp = bench.make_digest_workload(200_000, 0x6A, 2048, 0.25, 16)
    got, ref, grouped = grouped_vs_plain(ver, pub, sig, dig)
    assert grouped >= 1
    assert np.array_equal(got, exp) and np.array_equal(ref, exp)
    idx = np.random.default_rng(3).choice(len(exp), 4000, replace=False)
    assert np.array_equal(O.verify_digests(pub[idx], sig[idx], dig[idx], threads=16), got[idx])


def test_rejected_keys_repeated_across_the_batch(ver):
    """Goldens (every rejection class, infinity, x in [n, p), exceptional adds)
    tiled 300 times: 549 distinct keys over ~165k items."""
    gp, gs, gd, gok, _ = load_digest_vectors()
    reps = 300
    pub, sig, dig = (np.tile(a, (reps, 1)) for a in (gp, gs, gd))
    perm = np.random.default_rng(5).permutation(len(pub))
    pub, sig, dig = pub[perm], sig[perm], dig[perm]
    exp = np.tile(gok, reps)[perm]
    got, ref, grouped = grouped_vs_plain(ver, pub, sig, dig)
    assert grouped >= 1
    assert np.array_equal(got, exp) and np.array_equal(ref, exp)


def test_unique_keys_keep_the_pub33_route(ver):
    pub, sig, dig, exp = bench.make_digest_workload(100_000, 0x6B, 100_000, 0.0, 16)
    got, ref, grouped = grouped_vs_plain(ver, pub, sig, dig)
    assert grouped == 0
    assert np.array_equal(got, exp)


def test_grouped_device_resident_and_message_path(ver):
    n = 131_072
    pub, sig, dig, exp = bench.make_digest_workload(n, 0x6C, 1024, 0.25, 16)
    d = [ver.dev_alloc(a.nbytes) for a in (pub, sig, dig)]
    d_bits = ver.dev_alloc(((n + 63) // 64) * 8)
    for p, a in zip(d, (pub, sig, dig)):
        ver.dev_upload(p, a)
    b0, _ = ver.group_stats()
    for _ in range(3):                           # pipelined consecutive calls on the context stream
        ver.dev_verify_digests(0, n, d[0], d[1], d[2], d_bits)
    ver.dev_sync()
    bits = np.zeros((n + 63) // 64, np.uint64)
    ver.dev_download(bits, d_bits)
    assert np.array_equal(bench.unpack_bits(bits, n), exp)
    assert ver.group_stats()[0] - b0 == 3
    for p in d + [d_bits]:
        ver.dev_free(p)
    # message path: sign bytes hashed on the GPU, keys grouped
    from golden_io import load_msg_vectors
    mp, ms, mm, mok, _ = load_msg_vectors()
    reps = 400
    pub, sig = np.tile(mp, (reps, 1)), np.tile(ms, (reps, 1))
    msgs = mm * reps
    got, ref, grouped = grouped_vs_plain(ver, pub, sig, None, msgs=msgs)
    assert grouped >= 1 and np.array_equal(got, np.tile(mok, reps)) and np.array_equal(ref, got)


def test_host_slice_grouped_once_for_all_chunks(ver):
    """Host-buffer batches past the pipeline bound: the slice's keys are sent
    and grouped ONCE (slice_group), every chunk then runs keyed with the slots
    on the device -- pageable and pinned inputs, digests and messages, and a
    unique-key slice that must keep the per-chunk pub33 route."""
    pub, sig, dig, exp = bench.make_digest_workload(600_000, 0x6D, 4096, 0.25, 16)
    b0, _ = ver.group_stats()
    got = ver.verify_batch_digests(pub, sig, dig)
    b1, k1 = ver.group_stats()
    assert b1 - b0 == 1                          # one grouping for the whole slice, not one per chunk
    assert np.array_equal(got, exp)
    hp = [ver.host_array(a.shape, a.dtype) for a in (pub, sig, dig)]
    for h, a in zip(hp, (pub, sig, dig)):
        h[...] = a
    bits = ver.verify_batch_digests_bits(*hp)
    for h in hp:
        ver.host_free(h)
    assert ver.group_stats()[0] - b1 == 1
    assert np.array_equal(bench.unpack_bits(bits, len(exp)), exp)
    idx = np.random.default_rng(7).choice(len(exp), 3000, replace=False)
    assert np.array_equal(O.verify_digests(pub[idx], sig[idx], dig[idx], threads=16), got[idx])
    # message path: goldens tiled (every rejection class), shuffled
    from golden_io import load_msg_vectors
    mp, ms, mm, mok, _ = load_msg_vectors()
    reps = max(1, 200_000 // len(mp))
    perm = np.random.default_rng(8).permutation(reps * len(mp))
    pub2, sig2 = np.tile(mp, (reps, 1))[perm], np.tile(ms, (reps, 1))[perm]
    msgs = [(mm * reps)[i] for i in perm]
    b2, _ = ver.group_stats()
    got2 = ver.verify_batch_msgs(pub2, sig2, msgs)
    assert ver.group_stats()[0] - b2 == 1
    assert np.array_equal(got2, np.tile(mok, reps)[perm])
    # unique keys: no slice grouping
    pub3, sig3, dig3, exp3 = bench.make_digest_workload(300_000, 0x6E, 300_000, 0.1, 16)
    b3, _ = ver.group_stats()
    assert np.array_equal(ver.verify_batch_digests(pub3, sig3, dig3), exp3)
    assert ver.group_stats()[0] == b3


def test_host_slice_plain_first_chunk(ver):
    """gv_set_option("slice_plain_first"): a grouped host slice's first chunk
    runs the per-item pipeline while the slice's key tables build; the
    verdicts are the same, the slice is still grouped once, and exactly one
    chunk takes the per-item route."""
    pub, sig, dig, exp = bench.make_digest_workload(600_000, 0x6F, 4096, 0.25, 16)
    ver.set_option("slice_plain_first", 65536)
    try:
        b0, _ = ver.group_stats()
        r0 = ver.route_stats()
        got = ver.verify_batch_digests(pub, sig, dig)
        r1 = ver.route_stats()
        assert ver.group_stats()[0] - b0 == 1
        assert (r1["pub33"] + r1["item_f"]) - (r0["pub33"] + r0["item_f"]) == 1
        assert np.array_equal(got, exp)
        hp = [ver.host_array(a.shape, a.dtype) for a in (pub, sig, dig)]
        for h, a in zip(hp, (pub, sig, dig)):
            h[...] = a
        bits = ver.verify_batch_digests_bits(*hp)
        for h in hp:
            ver.host_free(h)
        assert np.array_equal(bench.unpack_bits(bits, len(exp)), exp)
    finally:
        ver.set_option("slice_plain_first", 0)


@pytest.mark.parametrize("pieces", [1, 3, 8])
def test_pageable_chunks_staged_in_pieces(ver, pieces):
    """gv_set_option("stage_pieces"): large pageable chunks are staged in
    pieces, each piece's H2D behind its copy; same verdicts for grouped and
    unique-key slices, digest bytes and bitmaps."""
    pub, sig, dig, exp = bench.make_digest_workload(500_000, 0x73, 4096, 0.25, 16)
    pu, su, du, eu = bench.make_digest_workload(200_000, 0x74, 200_000, 0.1, 16)
    ver.set_option("stage_pieces", pieces)
    try:
        assert np.array_equal(ver.verify_batch_digests(pub, sig, dig), exp)
        assert np.array_equal(bench.unpack_bits(ver.verify_batch_digests_bits(pu, su, du), len(eu)), eu)
    finally:
        ver.set_option("stage_pieces", 2)
