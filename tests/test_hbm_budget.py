"""A device whose HBM budget does not hold the optional tables must degrade to
a schedule that needs less, with the same verdicts (VERDICT r4 "make device
memory explicit"; DESIGN.md §7 HBM budget).

The budget is the library's own accounting of its optional device tables
(env GV_HBM_BUDGET_MB read by gv_open, or gv_set_option "hbm_budget_mb"):
the full-scalar G tables (6 GiB), the k6 G tables (3.5 GiB), k4's group G
tables (192 MiB), the per-batch grouping arenas and the resident key arena.
A real MI355X holds all of them, so the test shrinks the budget instead of
the device:

  budget     what fits                         grouped C2 batch     cached keys
  1 MiB      nothing optional                  per-item pub33       keys_load -> GV_ENOMEM
  1 GiB      k4 group G tables, small arenas   k4 (GLV G windows)   k4
  8 GiB      + full-scalar G tables            k4f                  k4f (no k6 tables)
  default    everything                        k4f                  kw (the arena's wide tables),
                                                                    kn (its k6 tables)
"""
import os

import numpy as np
import pytest

import bench
import gpuverify as gvm
from golden_io import load_digest_vectors

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def batch():
    pub, sig, dig, exp = bench.make_digest_workload(60_000, 0x93, 1024, 0.25, 16)
    gp, gs, gd, gok, _ = load_digest_vectors()
    pub, sig, dig = (np.concatenate([a, np.tile(b, (20, 1))]) for a, b in ((pub, gp), (sig, gs), (dig, gd)))
    exp = np.concatenate([exp, np.tile(gok, 20)])
    perm = np.random.default_rng(31).permutation(len(exp))
    return pub[perm], sig[perm], dig[perm], exp[perm]


def open_with_budget(mb):
    old = os.environ.get("GV_HBM_BUDGET_MB")
    os.environ["GV_HBM_BUDGET_MB"] = str(mb)
    try:
        return gvm.Verifier([0])
    finally:
        if old is None:
            del os.environ["GV_HBM_BUDGET_MB"]
        else:
            os.environ["GV_HBM_BUDGET_MB"] = old


def routes_of(ver, fn):
    r0 = ver.route_stats()
    out = fn()
    r1 = ver.route_stats()
    return out, {k: r1[k] - r0[k] for k in r1 if r1[k] != r0[k]}


@pytest.mark.parametrize("mb, grouped_route, keyed_route", [
    (1, "pub33", None),
    (1024, "k4", "k4"),
    (8192, "k4f", "k4f"),
])
def test_budget_degrades_with_the_same_verdicts(batch, mb, grouped_route, keyed_route):
    pub, sig, dig, exp = batch
    ver = open_with_budget(mb)
    try:
        got, routes = routes_of(ver, lambda: ver.verify_batch_digests(pub, sig, dig))
        assert np.array_equal(got, exp)
        assert routes.get(grouped_route, 0) >= 1, routes
        # device-resident (the bench's entry point) on the same batch
        n = len(exp)
        d = [ver.dev_alloc(a.nbytes) for a in (pub, sig, dig)]
        for p, a in zip(d, (pub, sig, dig)):
            ver.dev_upload(p, a)
        d_bits = ver.dev_alloc(((n + 63) // 64) * 8)
        ver.dev_verify_digests(0, n, d[0], d[1], d[2], d_bits)
        ver.dev_sync()
        bits = np.zeros((n + 63) // 64, np.uint64)
        ver.dev_download(bits, d_bits)
        assert np.array_equal(np.unpackbits(bits.view(np.uint8), bitorder="little")[:n], exp)
        for p in d + [d_bits]:
            ver.dev_free(p)
        uniq, inv = np.unique(pub, axis=0, return_inverse=True)
        if keyed_route is None:
            with pytest.raises(gvm.GpuVerifyError):
                ver.keys_load(uniq)
            return
        slots = ver.keys_load(uniq)[inv.reshape(-1)].astype(np.uint32)
        got2, routes2 = routes_of(ver, lambda: ver.verify_batch_digests_keyed(slots, sig, dig))
        assert np.array_equal(got2, exp)
        assert routes2.get(keyed_route, 0) >= 1, routes2
    finally:
        ver.close()


def test_default_budget_takes_the_arena_wide_then_k6_tables(batch):
    pub, sig, dig, exp = batch
    ver = gvm.Verifier([0])
    try:
        got, routes = routes_of(ver, lambda: ver.verify_batch_digests(pub, sig, dig))
        assert np.array_equal(got, exp)
        assert routes.get("k4f" if gvm.Verifier.KG_DEFAULT == 0 else "kg", 0) >= 1, routes   # the grouped default
        uniq, inv = np.unique(pub, axis=0, return_inverse=True)
        slots = ver.keys_load(uniq)[inv.reshape(-1)].astype(np.uint32)
        got, routes = routes_of(ver, lambda: ver.verify_batch_digests_keyed(slots, sig, dig))
        assert np.array_equal(got, exp)
        assert routes.get("kw", 0) >= 1, routes
        ver.set_option("keys_wide", 0)                  # the k6 tables of the same slots
        got, routes = routes_of(ver, lambda: ver.verify_batch_digests_keyed(slots, sig, dig))
        assert np.array_equal(got, exp)
        assert routes.get("kn", 0) >= 1, routes
    finally:
        ver.close()
