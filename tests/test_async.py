"""Asynchronous host batches (gv_submit_* / gv_wait, include/gpuverify.h):
batches queued back to back run as one stream of chunks per device -- the
next batch's staging, key grouping and key tables under the previous batch's
last chunks -- and must give exactly the synchronous entry points' verdicts,
whatever the mix of routes in the queue (grouped pub33, per-item pub33, keyed
slots, messages, small batches on the zero-copy kernels, pinned and pageable
buffers) and whatever the order of the waits."""
import gc

import numpy as np
import pytest

import bench
import gpuverify as gvm
from golden_io import load_digest_vectors, load_msg_vectors

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ver():
    v = gvm.Verifier([0])
    yield v
    v.close()


@pytest.fixture(scope="module")
def c2():
    return bench.make_digest_workload(300_000, 0x94, 4096, 0.25, 16)


def test_queue_of_mixed_batches_equals_synchronous(ver, c2):
    pub, sig, dig, exp = c2
    gp, gs, gd, gok, _ = load_digest_vectors()
    mp, ms, mm, mok, _ = load_msg_vectors()
    uniq, inv = np.unique(pub[:50_000], axis=0, return_inverse=True)
    ver.keys_reset()
    slots = ver.keys_load(uniq)[inv.reshape(-1)].astype(np.uint32)
    upub, usig, udig, uexp = bench.make_digest_workload(40_000, 0x95, 40_000, 0.2, 16)   # per-item route
    reps = 60
    tp, ts, td = (np.tile(x, (reps, 1)) for x in (gp, gs, gd))
    texp = np.tile(gok, reps)
    msgs = mm * 40
    mexp = np.tile(mok, 40)
    jobs = [
        (lambda: ver.submit_digests(pub, sig, dig), exp),                                  # grouped, 2 chunks
        (lambda: ver.submit_digests(upub, usig, udig), uexp),                              # per-item pub33
        (lambda: ver.submit_digests_keyed(slots, sig[:50_000], dig[:50_000]), exp[:50_000]),
        (lambda: ver.submit_digests(tp, ts, td), texp),                                    # goldens, tiled
        (lambda: ver.submit_digests(pub[:64], sig[:64], dig[:64]), exp[:64]),              # zero-copy small batch
        (lambda: ver.submit_msgs(np.tile(mp, (40, 1)), np.tile(ms, (40, 1)), msgs), mexp),  # message path
        (lambda: ver.submit_digests(pub[::-1].copy(), sig[::-1].copy(), dig[::-1].copy()), exp[::-1]),
    ]
    pend = [(f(), e) for f, e in jobs]
    # wait out of order: the last first, then the rest
    for p, e in [pend[-1]] + pend[:-1]:
        assert np.array_equal(ver.wait(p), e)
    ver.keys_reset()


def test_back_to_back_c2_batches_and_pinned_buffers(ver, c2):
    pub, sig, dig, exp = c2
    hp = [ver.host_array(a.shape, a.dtype) for a in (pub, sig, dig)]
    try:
        for h, a in zip(hp, (pub, sig, dig)):
            h[...] = a
        pend = [ver.submit_digests(*(hp if i % 2 else (pub, sig, dig))) for i in range(6)]
        for p in pend:
            assert np.array_equal(ver.wait(p), exp)
    finally:
        for h in hp:
            ver.host_free(h)


def test_tickets(ver, c2):
    pub, sig, dig, exp = c2
    p0 = ver.submit_digests(pub[:0], sig[:0], dig[:0])
    assert ver.wait(p0).shape == (0,)
    p = ver.submit_digests(pub[:1000], sig[:1000], dig[:1000])
    assert np.array_equal(ver.wait(p), exp[:1000])
    with pytest.raises(gvm.GpuVerifyError):                 # a ticket is waited for once
        ver.wait(p)
    with pytest.raises(gvm.GpuVerifyError):
        ver.wait(gvm.Verifier.Pending(123456789, None))


def test_keys_load_waits_for_submitted_keyed_batches(ver, c2):
    pub, sig, dig, exp = c2
    uniq, inv = np.unique(pub[:100_000], axis=0, return_inverse=True)
    ver.keys_reset()
    slots = ver.keys_load(uniq)[inv.reshape(-1)].astype(np.uint32)
    pend = [ver.submit_digests_keyed(slots, sig[:100_000], dig[:100_000]) for _ in range(3)]
    ver.keys_reset()                                         # returns only after the three batches ran
    ver.keys_load(pub[::-1][:4096])                           # other keys in the same slots
    for p in pend:
        assert np.array_equal(ver.wait(p), exp[:100_000])
    ver.keys_reset()


def test_sync_calls_interleave_with_the_queue(ver, c2):
    pub, sig, dig, exp = c2
    p1 = ver.submit_digests(pub, sig, dig)
    got = ver.verify_batch_digests(pub[:70_000], sig[:70_000], dig[:70_000])   # waits for the lane's device lock
    p2 = ver.submit_digests(pub, sig, dig)
    assert np.array_equal(got, exp[:70_000])
    assert np.array_equal(ver.wait(p2), exp)
    assert np.array_equal(ver.wait(p1), exp)


def test_dropped_pending_is_waited_before_its_buffers_go(ver, c2):
    """the library reads a batch's inputs and writes its verdicts
    until gv_wait.  A Pending dropped without wait() must not free them under
    the lane: the Verifier keeps them and waits for the ticket when the
    Pending is collected."""
    pub, sig, dig, exp = c2
    for k in range(3):                                        # fresh copies: nothing else holds them
        ver.submit_digests(pub.copy(), sig.copy(), dig.copy())
    gc.collect()
    assert not ver._inflight                                  # every dropped ticket was waited for
    p = ver.submit_digests(pub, sig, dig)
    assert np.array_equal(ver.wait(p), exp)


def test_close_waits_for_outstanding_batches(c2):
    pub, sig, dig, exp = c2
    v = gvm.Verifier([0])
    p = v.submit_digests(pub, sig, dig)
    v.close()                                                 # waits for the ticket, then gv_close
    assert np.array_equal(p.out, exp)


def test_pinned_batches_whole_or_chunked(c2):
    """Pinned batches queued behind one in flight run as one chunk
    ("async_whole", default), as fixed chunks (off), or -- past max_batch --
    as several max_batch chunks sharing one slice grouping; keyed pinned
    batches the same.  Same verdicts every way."""
    pub, sig, dig, exp = c2
    v = gvm.Verifier([0])
    hp = [v.host_array(a.shape, a.dtype) for a in (pub, sig, dig)]
    try:
        assert v.get_option("async_whole") == 1
        assert v.get_option("async_chunk") == 262144 and v.get_option("async_growth") == 1
        for h, a in zip(hp, (pub, sig, dig)):
            h[...] = a
        for whole, mb in ((1, None), (0, None), (1, 131072)):
            v.set_option("async_whole", whole)
            if mb:
                v.set_option("max_batch", mb)
            assert v.get_option("async_whole") == whole
            pend = [v.submit_digests(*hp) for _ in range(4)]
            for p in pend:
                assert np.array_equal(v.wait(p), exp)
        uniq, inv = np.unique(pub, axis=0, return_inverse=True)
        hs = v.host_array((len(pub),), np.uint32)
        try:
            hs[...] = v.keys_load(uniq)[inv.reshape(-1)].astype(np.uint32)
            pend = [v.submit_digests_keyed(hs, hp[1], hp[2]) for _ in range(3)]
            for p in pend:
                assert np.array_equal(v.wait(p), exp)
        finally:
            v.host_free(hs)
    finally:
        for h in hp:
            v.host_free(h)
        v.close()
