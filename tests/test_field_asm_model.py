"""CPU validation of the hand-scheduled gfx950 field sequences.

tools/gen_field_asm.py generates the inline-asm blocks of
cosmos-sdk-rootchain_amd/csrc/secp_field_asm.inc from instruction tuples and
also executes those tuples on an instruction-level model (VGPR/VCC semantics of
v_mad_u64_u32, v_addc_co_u32, v_subb_co_u32, v_alignbit_b32, ...).  This test
checks every sequence against Python integer arithmetic, checks that no carry
is read away from its writer (the back-to-back rule), and that the committed
.inc file is exactly what the generator produces."""
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import gen_field_asm as G  # noqa: E402

P = G.P
EDGE = [0, 1, 2, 977, 2**32 - 1, 2**32, P - 1, P, P + 1, 2**256 - 1, 2**256 - 2**32 - 978, 2**255,
        (2**32 - 1) << 224, int("FFFFFFFF" * 4 + "0" * 32, 16)]


def test_generated_include_is_current():
    path = os.path.join(REPO, "cosmos-sdk-rootchain_amd", "csrc", "secp_field_asm.inc")
    assert open(path).read() == G.generate()


def test_no_carry_hazards():
    for g in (G.gen_mul512, G.gen_sqr_cross, G.gen_sqr_finish, G.gen_reduce, G.gen_add, G.gen_sub, G.gen_mul3):
        assert G.hazard_check(g()) is None, g.__name__
    for s in (1, 2, 3):
        assert G.hazard_check(G.gen_shl(s)) is None
        assert G.hazard_check(G.gen_sub_shl(s)) is None


def test_sequences_match_integer_arithmetic():
    rng = random.Random(0xA5)
    vals = EDGE + [rng.randrange(2**256) for _ in range(1500)]
    for a in vals:
        b = rng.choice(vals)
        assert G.emu_mul512(a, b) == a * b
        assert G.emu_sqr(a) == a * a
        r = G.emu_add(a, b)
        assert r < 2**256 and r % P == (a + b) % P
        r = G.emu_sub(a, b)
        assert r < 2**256 and r % P == (a - b) % P
    for t in [0, 2**512 - 1, (2**256 - 1) ** 2, P * P, (P - 1) ** 2] + [rng.randrange(2**512) for _ in range(1500)]:
        r = G.emu_reduce(t)
        assert r < 2**256 and r % P == t % P


def test_shift_and_small_multiple_sequences():
    rng = random.Random(0x5A)
    vals = EDGE + [rng.randrange(2**256) for _ in range(800)]
    for a in vals:
        r = G.emu_mul3(a)
        assert r < 2**256 and r % P == 3 * a % P
        for s in (1, 2, 3):
            r = G.emu_shl(a, s)
            assert r < 2**256 and r % P == (a << s) % P
            for b in [rng.choice(vals)] + EDGE[-6:]:
                r = G.emu_sub_shl(a, b, s)
                assert r < 2**256 and r % P == (a - (b << s)) % P
