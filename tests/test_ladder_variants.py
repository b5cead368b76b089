"""The keyed ladder's schedules must agree bit for bit: the grouped route's
many-group 5-bit ladders (gv_set_option "kg" 6 / 7 / 9: k4's 16-entry tables
over 6, 7 or 9 groups, 20 / 15 / 10 doublings, G after the last doubling on the
real curve), k_ecmult_k4 with the G
half on the unsplit scalar (gv_set_option "gfull" 1, the default: 11 signed
25-bit windows of u1 from the 2^o G tables), k_ecmult_k4 on the GLV-split G
half (gfull 0: 14 20-bit windows) and k_ecmult_k6 (6-bit Q windows on 32-entry
key tables, the lambda frame, G on the unsplit u1 in 11 signed 24-bit windows
from the 2^(36 t) G tables: "k6" 1 on the grouped route, "keys_k6" 1 -- the
default -- on the resident key arena), and the arena's wide-window tables
("keys_wide", the default: 11-bit Q windows on 1,024-entry tables, one window per
group and no doublings, or two per group and 11 doublings).  Each is run on the grouped route (pub33
batches with repeated keys), the cached-key route (gv_keys_load slots) and the
message path, against the oracle's expected verdicts, and the route counters
must show the schedule that ran.  The per-item route (group_keys 0: each item parses its
key, 26 five-bit windows over 125 doublings) runs both its G schedules too:
"gfull_item" 1 (the default: u1's 11 25-bit windows from the same 2^o G
tables, windows past bit 125 from the 2^45 / 2^100 / 2^145 ones) and 0 (14
GLV windows)."""
import numpy as np
import pytest

import bench
import gpuverify as gvm
from golden_io import load_digest_vectors, load_msg_vectors
from oracle import oracle as O

pytestmark = pytest.mark.gpu

KG_DEFAULT = gvm.Verifier.KG_DEFAULT            # the library's default "kg" layout (0: k4 on the grouped route)
SCHEDULES = {"k4f": {"gfull": 1, "k6": 0, "kg": 0}, "k4": {"gfull": 0, "k6": 0, "kg": 0},
             "k6": {"gfull": 1, "k6": 1, "kg": 0},
             "kg4": {"kg": 4}, "kg6": {"kg": 6}, "kg7": {"kg": 7}, "kg9": {"kg": 9},
             "item_gf": {"group_keys": 0, "gfull_item": 1}, "item_glv": {"group_keys": 0, "gfull_item": 0}}
ROUTE = {"k4f": "k4f", "k4": "k4", "k6": "k6", "kg4": "kg", "kg6": "kg", "kg7": "kg", "kg9": "kg", "wide": "k6", "wide2": "k6",
         "item_gf": "item_f", "item_glv": "pub33"}
DEFAULTS = {"gfull": 1, "k6": 0, "kg": KG_DEFAULT, "group_keys": 1, "gfull_item": 1, "keys_k6": 1, "keys_wide": 2,
            "keys_wide1_cap": 0}
# the cached-key route (gv_keys_load slots): k6 / wide-window tables are built
# at load time when "keys_k6" / "keys_wide" are on; the message part of the test runs
# the grouped route
CACHED = {"k4f": {"gfull": 1, "keys_k6": 0, "keys_wide": 0, "k6": 0, "kg": 0},
          "k4": {"gfull": 0, "keys_k6": 0, "keys_wide": 0, "k6": 0, "kg": 0},
          "k6": {"gfull": 1, "keys_k6": 1, "keys_wide": 0, "k6": 1, "kg": 0},
          "wide": {"gfull": 1, "keys_k6": 1, "keys_wide": 2, "k6": 1, "kg": 0},
          "wide2": {"gfull": 1, "keys_k6": 1, "keys_wide": 1, "k6": 1, "kg": 0}}
ARENA_ROUTE = {"k6": "kn", "wide": "kw", "wide2": "kw2"}          # schedule -> the arena's route counter


@pytest.fixture(scope="module")
def ver():
    v = gvm.Verifier([0])
    yield v
    for k, val in DEFAULTS.items():
        v.set_option(k, val)
    v.close()


def run(ver, sched, fn, table=None):
    for k, val in (table or SCHEDULES)[sched].items():
        ver.set_option(k, val)
    r0 = ver.route_stats()
    try:
        out = fn()
    finally:
        for k, val in DEFAULTS.items():
            ver.set_option(k, val)
    r1 = ver.route_stats()
    d = {k: r1[k] - r0[k] for k in r1}
    return out, dict(d, **{sched: d[ROUTE[sched]]})


@pytest.mark.parametrize("sched", list(SCHEDULES))
def test_grouped_random_with_adversarial(ver, sched):
    pub, sig, dig, exp = bench.make_digest_workload(70_001, 0x91, 1500, 0.25, 16)
    got, routes = run(ver, sched, lambda: ver.verify_batch_digests(pub, sig, dig))
    assert routes[sched] >= 1, routes
    assert np.array_equal(got, exp)
    idx = np.random.default_rng(21).choice(len(exp), 2000, replace=False)
    assert np.array_equal(O.verify_digests(pub[idx], sig[idx], dig[idx], threads=16), got[idx])


@pytest.mark.parametrize("sched", list(SCHEDULES))
def test_grouped_goldens_tiled(ver, sched):
    """every rejection class and the exceptional-add vectors, tiled and shuffled"""
    gp, gs, gd, gok, _ = load_digest_vectors()
    reps = 100
    perm = np.random.default_rng(22).permutation(reps * len(gp))
    pub, sig, dig = (np.tile(x, (reps, 1))[perm] for x in (gp, gs, gd))
    exp = np.tile(gok, reps)[perm]
    got, routes = run(ver, sched, lambda: ver.verify_batch_digests(pub, sig, dig))
    assert routes[sched] >= 1, routes
    assert np.array_equal(got, exp)


P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def ec_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if (a[1] + b[1]) % P == 0:
            return None
        lam = 3 * a[0] * a[0] * pow(2 * a[1], -1, P) % P
    else:
        lam = (b[1] - a[1]) * pow(b[0] - a[0], -1, P) % P
    x = (lam * lam - a[0] - b[0]) % P
    return x, (lam * (a[0] - x) - a[1]) % P


def forge(pub, u1, rng):
    """(sig, digest) that verifies under pub with e/s = u1 exactly: R = u1 G +
    u2 Q for a random u2, r = R.x mod n, s = r/u2 (retried until low-S), e = u1 s"""
    while True:
        u2 = int(rng.integers(1, 1 << 62)) * int(rng.integers(1, 1 << 62)) % N or 1
        R = ec_add(O.point_mul(u1) if u1 else None, O.point_mul(u2, pub))
        if R is None or R[0] % N == 0:
            continue
        r = R[0] % N
        s = r * pow(u2, -1, N) % N
        if s > N // 2:
            continue
        e = u1 * s % N
        return r.to_bytes(32, "big") + s.to_bytes(32, "big"), e.to_bytes(32, "big")


def test_scalar_edges_on_the_full_scalar_windows(ver):
    """u1 = e/s on the edges of the 25-bit G windows (0, 1, n - 1, every
    digit at +-2^24, the top window's carry, all-ones patterns), forged so
    they verify, plus the same signatures under the wrong key"""
    rng = np.random.default_rng(24)
    keys = [O.pubkey(O.privkey_from_secret(b"ladder-variants-%d" % i)) for i in range(8)]
    top = sum(1 << (25 * j + 24) for j in range(10))           # every window's top bit: digits -2^24 (+carry)
    low = sum(((1 << 24) - 1) << (25 * j) for j in range(10))  # low 24 bits ones, no borrow
    top6 = sum(1 << (24 * j + 23) for j in range(10))          # the same for k6's 24-bit windows
    low6 = sum(((1 << 23) - 1) << (24 * j) for j in range(10))
    u1s = [0, 1, 2, N - 1, N - 2, (1 << 24), (1 << 24) - 1, (1 << 24) + 1, top % N, (top | low) % N,
           low % N, ((1 << 256) - 1) % N, (1 << 255) % N, ((1 << 250) - 1) % N, (N - 1) >> 1,
           (1 << 23), (1 << 23) - 1, (1 << 23) + 1, top6 % N, (top6 | low6) % N, low6 % N, (1 << 240) % N]
    pubs, sigs, digs = [], [], []
    for u1 in u1s:
        for qi, q in enumerate(keys):
            sg, dg = forge(q, u1, rng)
            pubs += [q, keys[(qi + 1) % len(keys)]]
            sigs += [sg, sg]
            digs += [dg, dg]
    m = len(pubs)
    pub = np.frombuffer(b"".join(pubs), np.uint8).reshape(m, 33)
    sig = np.frombuffer(b"".join(sigs), np.uint8).reshape(m, 64)
    dig = np.frombuffer(b"".join(digs), np.uint8).reshape(m, 32)
    want = O.verify_digests(pub, sig, dig, threads=16)
    assert want[0::2].all() and not want[1::2].any()
    reps = 60                                                   # 21,120 items on 8 keys: the grouped route
    pub, sig, dig = (np.tile(x, (reps, 1)) for x in (pub, sig, dig))
    exp = np.tile(want, reps)
    for sched in SCHEDULES:
        got, routes = run(ver, sched, lambda: ver.verify_batch_digests(pub, sig, dig))
        assert routes[sched] >= 1, (sched, routes)
        assert np.array_equal(got, exp), sched


@pytest.mark.parametrize("sched", list(CACHED))
def test_cached_keys_and_messages(ver, sched):
    for k, val in CACHED[sched].items():                       # keys_k6 decides which tables the load builds
        ver.set_option(k, val)
    ver.keys_reset()
    pub, sig, dig, exp = bench.make_digest_workload(40_000, 0x92, 300, 0.25, 16)
    uniq, inv = np.unique(pub, axis=0, return_inverse=True)
    slots = ver.keys_load(uniq)[inv.reshape(-1)].astype(np.uint32)
    got, routes = run(ver, sched, lambda: ver.verify_batch_digests_keyed(slots, sig, dig), CACHED)
    assert routes[ARENA_ROUTE.get(sched, sched)] >= 1, routes   # the arena's k6 (11 groups) / wide (8 groups) tables
    assert np.array_equal(got, exp)
    mp, ms, mm, mok, _ = load_msg_vectors()
    reps = max(1, 40_000 // len(mp))
    perm = np.random.default_rng(23).permutation(reps * len(mp))
    pub2, sig2 = np.tile(mp, (reps, 1))[perm], np.tile(ms, (reps, 1))[perm]
    msgs = [(mm * reps)[i] for i in perm]
    got2, routes = run(ver, sched, lambda: ver.verify_batch_msgs(pub2, sig2, msgs), CACHED)
    assert routes[sched] >= 1, routes
    assert np.array_equal(got2, np.tile(mok, reps)[perm])


def test_cached_keys_k6_goldens_and_slots(ver):
    """k6 on the resident arena: the golden rejection classes loaded as keys
    (ParsePubKey rejects get a slot too) tiled over a throughput batch,
    out-of-range slots, a second load appended to the arena (the k6 tables of
    both loads), all against the k4 route on the same slots"""
    gp, gs, gd, gok, _ = load_digest_vectors()
    ver.keys_reset()
    half = len(gp) // 2
    s1 = ver.keys_load(gp[:half])
    s2 = ver.keys_load(gp[half:])                                 # appended: slots half..
    slots_g = np.concatenate([s1, s2]).astype(np.uint32)
    reps = 150
    perm = np.random.default_rng(25).permutation(reps * len(gp))
    slots = np.tile(slots_g, reps)[perm]
    sig, dig = np.tile(gs, (reps, 1))[perm], np.tile(gd, (reps, 1))[perm]
    exp = np.tile(gok, reps)[perm].copy()
    bad = np.random.default_rng(26).random(len(slots)) < 0.01     # slots past the arena: never valid
    slots[bad] = len(gp) + 7
    exp[bad] = 0
    got6, r6 = run(ver, "k6", lambda: ver.verify_batch_digests_keyed(slots, sig, dig), CACHED)
    assert r6["kn"] >= 1, r6
    assert np.array_equal(got6, exp)
    gotw, rw = run(ver, "wide", lambda: ver.verify_batch_digests_keyed(slots, sig, dig), CACHED)
    assert rw["kw"] >= 1, rw
    assert np.array_equal(gotw, exp)
    ver.set_option("keys_k6", 0)                                  # the k4 tables of the same slots
    try:
        got4, r4 = run(ver, "k4f", lambda: ver.verify_batch_digests_keyed(slots, sig, dig), CACHED)
    finally:
        ver.set_option("keys_k6", 1)
    assert r4["k4f"] >= 1, r4
    assert np.array_equal(got4, got6)
    ver.keys_reset()


@pytest.mark.parametrize("layout", ["one", "two", "relayout"])
def test_wide_arena_growth_keeps_the_loaded_slots(ver, layout):
    """The wide-window tables live in an arena of their own that grows by
    doubling from 4,096 slots: a second load past it copies the first load's
    tables into the grown arena (Z rows re-strided) and builds the rest; every
    slot then verifies on the wide-window ladder exactly as on the k6 one, and
    a load after gv_keys_reset rebuilds from slot 0.  Layouts: one window per
    group (keys_wide 2), two (keys_wide 1), and one window per group whose
    growth is refused (keys_wide1_cap 4,096): the whole arena moves to two
    windows per group, the first load's keys read back from the k4 tables."""
    pub, sig, dig, exp = bench.make_digest_workload(30_000, 0x98, 6000, 0.25, 16)
    want = O.verify_digests(pub, sig, dig, threads=16)
    route = "kw" if layout == "one" else "kw2"
    sched = "wide" if layout != "two" else "wide2"
    ver.keys_reset()
    ver.set_option("keys_wide", 1 if layout == "two" else 2)
    ver.set_option("keys_wide1_cap", 4096 if layout == "relayout" else 0)
    try:
        uniq, first, inv = np.unique(pub, axis=0, return_index=True, return_inverse=True)
        order = np.argsort(first)
        a = ver.keys_load(uniq[order][:3000])
        b = ver.keys_load(uniq[order][3000:])                      # past 4,096 slots: the wide arena grows
        slots_u = np.concatenate([a, b]).astype(np.uint32)
        rank = np.empty_like(order)
        rank[order] = np.arange(len(order))
        slots = slots_u[rank[inv.reshape(-1)]]
        gotw, rw = run(ver, sched, lambda: ver.verify_batch_digests_keyed(slots, sig, dig), CACHED)
        assert rw[route] >= 1, rw
        assert np.array_equal(gotw, want)
        got6, r6 = run(ver, "k6", lambda: ver.verify_batch_digests_keyed(slots, sig, dig), CACHED)
        assert r6["kn"] >= 1, r6
        assert np.array_equal(got6, want)
        ver.set_option("keys_wide", 1 if layout == "two" else 2)
        ver.set_option("keys_wide1_cap", 4096 if layout == "relayout" else 0)
        ver.keys_reset()                                           # slots rewritten from 0
        c = ver.keys_load(uniq[order][3000:]).astype(np.uint32)
        sub = rank[inv.reshape(-1)] >= 3000
        s2 = c[rank[inv.reshape(-1)][sub] - 3000]
        got, r = run(ver, sched, lambda: ver.verify_batch_digests_keyed(s2, sig[sub], dig[sub]), CACHED)
        assert r["kw" if layout == "one" else "kw2"] >= 1 or (layout == "relayout" and r["kw"] >= 1), r
        assert np.array_equal(got, want[sub])
    finally:
        ver.set_option("keys_wide", 2)
        ver.set_option("keys_wide1_cap", 0)
        ver.keys_reset()
