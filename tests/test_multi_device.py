"""The node-shaped multi-GPU path: ONE context over several
devices, host batches split into contiguous per-device slices on persistent
workers, staging through ONE pool shared by all devices, bitmaps gathered.

* two DISTINCT device ids (skipped when only one device is visible -- the
  round's GPU box has one; the 8-GPU node runs bench.py --inproc);
* one device opened as two slots, driven from concurrent threads: the shared
  staging pool takes overlapping jobs from both slices and from both callers.
Verdicts against the construction and the C oracle on a sample."""
import threading

import numpy as np
import pytest

import bench
import gpuverify as gvm
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def workload(n, seed):
    return bench.make_digest_workload(n, seed, 4096, 0.25, 16)


def visible_devices():
    v = gvm.Verifier()
    n = v.num_devices
    v.close()
    return n


def test_two_distinct_devices_split_and_gather():
    if visible_devices() < 2:
        pytest.skip("one visible device")
    pub, sig, dig, exp = workload(600_000, 0xD1)
    with gvm.Verifier([0, 1]) as v:
        got = v.verify_batch_digests(pub, sig, dig)
        sl = v.last_slices()
        bits = v.verify_batch_digests_bits(pub, sig, dig)
    assert np.array_equal(got, exp)
    assert np.array_equal(bench.unpack_bits(bits, len(exp)), exp)
    assert len(sl) == 2 and all(c > 0 and ms > 0 for ms, c in sl) and sum(c for _, c in sl) == len(exp)
    idx = np.random.default_rng(1).choice(len(exp), 5000, replace=False)
    assert np.array_equal(O.verify_digests(pub[idx], sig[idx], dig[idx], threads=16), got[idx])


def test_shared_staging_pool_under_concurrent_callers():
    """Two device slots of one context, two caller threads, host batches large
    enough to take the pipelined staging path: every verdict as constructed."""
    batches = [workload(400_000, 0xD2 + i) for i in range(2)]
    out = [None, None]
    with gvm.Verifier([0, 0]) as v:
        def run(i):
            p, s, d, _ = batches[i]
            out[i] = [v.verify_batch_digests(p, s, d) for _ in range(2)]
        th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        sl = v.last_slices()
    for i in range(2):
        for got in out[i]:
            assert np.array_equal(got, batches[i][3])
    assert len(sl) == 2 and all(c > 0 for _, c in sl)


@pytest.mark.parametrize("n", [1, 700, 5000, 300_000])
def test_pinned_caller_buffers(n):
    """Caller arrays in pinned memory (gv_host_alloc) skip the staging copy:
    small batches read them in place (sliced kernels), large ones copy them
    straight to the device.  Same verdicts as pageable arrays."""
    pub, sig, dig, exp = bench.make_digest_workload(n, 0xD7 + n, 4096, 0.25, 16)
    with gvm.Verifier([0]) as v:
        hp = [v.host_array(a.shape, a.dtype) for a in (pub, sig, dig)]
        for h, a in zip(hp, (pub, sig, dig)):
            h[...] = a
        got = v.verify_batch_digests(*hp)
        again = v.verify_batch_digests(pub, sig, dig)
        for h in hp:
            v.host_free(h)
    assert np.array_equal(got, exp) and np.array_equal(again, exp)
