"""The full-scalar G schedule of k_ecmult_k4<true> (gv_kernels.hip kGFOff /
kGFWin / kGFTab, gv_kernels.h GV_GF_*), checked on the CPU from the kernel
source's own constants:

* every window j in 0..GV_GF_WIN-1 is added exactly once, at one ladder
  position p in 0..6, from the table of offset 25 j - 5 p (the accumulator
  is doubled 5 p more times after position p, so the entry d * 2^off * G
  lands at d * 2^(25 j) * G);
* a table holds at most the windows its 2^24 signed digits can serve;
* the signed 25-bit Booth recoding (booth_digit8: digit j from bits
  25 j - 1 .. 25 j + 24, in [-2^24, 2^24]) of any u1 < n sums back to u1
  and never indexes past the 2^24-entry tables, and the ladder's positions
  put the windows back together into u1.
"""
import os
import random
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = open(os.path.join(REPO, "cosmos-sdk-rootchain_amd", "csrc", "gv_kernels.hip")).read()
HDR = open(os.path.join(REPO, "cosmos-sdk-rootchain_amd", "csrc", "gv_kernels.h")).read()
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def define(name):
    return int(re.search(r"#define " + name + r" \(?(\d+)", HDR).group(1))


def array(name):
    body = re.search(name + r"\[[^\]]*\](?:\[[^\]]*\])? = \{(.*?)\};", SRC, re.S).group(1)
    return [int(x) for x in re.findall(r"-?\d+", body)]


W, WIN, NTAB = define("GV_GF_W"), define("GV_GF_WIN"), define("GV_GF_NTAB")
OFF = array("kGFOff")
WINS = array("kGFWin")           # 7 positions x 4 slots, -1 = none
TAB = array("kGFTab")


def booth(k, j):
    p = W * j - 1
    v = (k << 1) & ((1 << (W + 1)) - 1) if p < 0 else (k >> p) & ((1 << (W + 1)) - 1)
    mag = ((v >> 1) & ((1 << (W - 1)) - 1)) + (v & 1)
    return mag - ((v >> W) << (W - 1))


def test_constants_shape():
    assert (W, WIN, NTAB) == (25, 11, 6)
    assert len(OFF) == NTAB and len(TAB) == WIN and len(WINS) == 7 * 4
    assert W * WIN >= 257


def test_every_window_once_at_its_offset():
    seen = {}
    for p in range(7):
        for j in WINS[4 * p:4 * p + 4]:
            if j < 0:
                continue
            assert j not in seen, f"window {j} added twice"
            seen[j] = p
            assert OFF[TAB[j]] == W * j - 5 * p, (j, p, TAB[j])
    assert sorted(seen) == list(range(WIN))
    for t in range(NTAB):                          # each table serves windows at its offset's positions only
        assert all(OFF[t] <= W * j <= OFF[t] + 30 for j in range(WIN) if TAB[j] == t)


def test_booth_windows_reconstruct_u1_within_table_range():
    rng = random.Random(7)
    vals = [0, 1, 2, N - 1, N - 2, (1 << 24), (1 << 24) - 1, (1 << 255) % N, ((1 << 256) - 1) % N]
    vals += [rng.randrange(N) for _ in range(2000)]
    for u1 in vals:
        d = [booth(u1, j) for j in range(WIN)]
        assert sum(dj << (W * j) for j, dj in enumerate(d)) == u1
        assert all(-(1 << (W - 1)) <= dj <= (1 << (W - 1)) for dj in d)
        assert all(abs(dj) - 1 < (1 << (W - 1)) for dj in d if dj)     # entry |d| - 1 < GV_GF_TAB_N


def test_ladder_positions_reconstruct_the_g_scalar():
    """sum over positions p of (sum of the position's entries) * 2^(5p) ==
    u1 -- what the 30-doubling accumulator computes for the G half."""
    rng = random.Random(11)
    for _ in range(500):
        u1 = rng.randrange(N)
        total = 0
        for p in range(7):
            for j in WINS[4 * p:4 * p + 4]:
                if j >= 0:
                    total += (booth(u1, j) << OFF[TAB[j]]) << (5 * p)
        assert total == u1
