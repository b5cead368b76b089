#!/usr/bin/env python3
"""Generate cosmos-sdk-rootchain_amd/csrc/secp_field_asm.inc -- the hand-scheduled
gfx950 inline-asm sequences of the secp256k1 field layer -- and emulate them.

Why asm: hipcc interleaves unrelated moves into __builtin_addc carry chains and
then pads every VCC read that is one instruction away from its VCC write with
an `s_nop 0` (measured: 228 nops in one point doubling).  Each sequence below
keeps every carry chain strictly back-to-back (a VCC/SGPR-carry write is read
by the very next instruction or not at all), so no wait states are needed.

Sequences (operands are named; v0..v3 and VCC are clobbered scratch):
  MUL512  t[16] = a[8] * b[8]             product scanning, 2 ops / product
  SQRX    c[16] = sum_{i<j} a_i a_j 2^(32(i+j))   cross products only
  SQRF    t[16] = 2*c + sum_i (sqlo_i + sqhi_i 2^32) 2^(64 i)
  RED     r[8]  = t (512-bit) mod p, weakly reduced (< 2^256)
  ADD     r[8]  = a + b mod p (weak),   SUB  r[8] = a - b mod p (weak)

The emulator (class Machine) executes the same instruction tuples on Python
ints; tests/test_field_asm_model.py checks every sequence on random and edge
inputs, so a schedule error is caught on the CPU before a GPU run.
"""
import os

M32 = 0xFFFFFFFF
P = 2**256 - 2**32 - 977


# ------------------------------------------------------------------ program
class Prog:
    def __init__(self):
        self.ins = []

    def __call__(self, op, *args):
        self.ins.append((op,) + args)


def vreg(i):
    return f"v{i}"


def pair(i):
    return f"v[{i}:{i + 1}]"


# Operand naming: "%[name]" for compiler-allocated operands; v0..v3 scratch.
def gen_mul512():
    p = Prog()
    pairs = [(0, 1), (2, 3)]
    for k in range(15):
        P_, Q_ = pairs[k % 2], pairs[(k + 1) % 2]
        prods = [(i, k - i) for i in range(8) if 0 <= k - i < 8]
        first = True
        for (i, j) in prods:
            if k == 0:
                p("mad", pair(P_[0]), "vcc", f"%[a{i}]", f"%[b{j}]", "0")
                p("mov", vreg(Q_[1]), "0")
                continue
            p("mad", pair(P_[0]), "vcc", f"%[a{i}]", f"%[b{j}]", pair(P_[0]))
            if k == 14:
                continue
            if first:
                p("addc", vreg(Q_[1]), "vcc", "0", "0", "vcc")
                first = False
            else:
                p("addc", vreg(Q_[1]), "vcc", "0", vreg(Q_[1]), "vcc")
        p("mov", f"%[t{k}]", vreg(P_[0]))
        if k < 14:
            p("mov", vreg(Q_[0]), vreg(P_[1]))
        else:
            p("mov", "%[t15]", vreg(P_[1]))
    return p


def gen_sqr_cross():
    """c1..c15 (c0 == 0 is not produced) = cross products a_i a_j, i < j."""
    p = Prog()
    pairs = [(0, 1), (2, 3)]
    started = False
    for k in range(1, 14):
        P_, Q_ = pairs[k % 2], pairs[(k + 1) % 2]
        prods = [(i, k - i) for i in range(8) if i < k - i <= 7]
        first = True
        for (i, j) in prods:
            if not started:
                p("mad", pair(P_[0]), "vcc", f"%[a{i}]", f"%[a{j}]", "0")
                p("mov", vreg(Q_[1]), "0")
                started = True
                continue
            p("mad", pair(P_[0]), "vcc", f"%[a{i}]", f"%[a{j}]", pair(P_[0]))
            if first:
                p("addc", vreg(Q_[1]), "vcc", "0", "0", "vcc")
                first = False
            else:
                p("addc", vreg(Q_[1]), "vcc", "0", vreg(Q_[1]), "vcc")
        p("mov", f"%[c{k}]", vreg(P_[0]))
        if k < 13:
            p("mov", vreg(Q_[0]), vreg(P_[1]))
        else:
            # the cross sum is < 2^511, so c15 (the last carry count) may be nonzero
            p("mov", "%[c14]", vreg(P_[1]))
            p("mov", "%[c15]", vreg(Q_[1]))
    return p


def gen_sqr_finish():
    """t = 2c + S, c = c1..c15 (c0 = 0), S_{2i} = sqlo_i, S_{2i+1} = sqhi_i."""
    p = Prog()
    # pass 1: doubled cross limbs d_k = (c_k << 1) | (c_{k-1} >> 31) into t_k
    p("mov", "%[t0]", "%[sl0]")
    p("lshl1", "%[t1]", "%[c1]")
    for k in range(2, 16):
        p("alignbit", f"%[t{k}]", f"%[c{k}]", f"%[c{k - 1}]", "31")
    # pass 2: one back-to-back carry chain adding the squares
    p("add_co", "%[t1]", "vcc", "%[t1]", "%[sh0]")
    for i in range(1, 8):
        p("addc", f"%[t{2 * i}]", "vcc", f"%[t{2 * i}]", f"%[sl{i}]", "vcc")
        p("addc", f"%[t{2 * i + 1}]", "vcc", f"%[t{2 * i + 1}]", f"%[sh{i}]", "vcc")
    return p


def gen_reduce():
    """r = L + H*977 + (H << 32), folded twice.  mlo_i/mhi_i = halves of H_i*977."""
    p = Prog()
    # chain A: r = L + mlo ; top = mhi7 + carry
    p("add_co", "%[r0]", "vcc", "%[t0]", "%[ml0]")
    for i in range(1, 8):
        p("addc", f"%[r{i}]", "vcc", f"%[t{i}]", f"%[ml{i}]", "vcc")
    p("addc", "%[top]", "vcc", "%[mh7]", "0", "vcc")
    # chain B: r[1..7] += mhi[0..6] ; top += carry
    p("add_co", "%[r1]", "vcc", "%[r1]", "%[mh0]")
    for i in range(2, 8):
        p("addc", f"%[r{i}]", "vcc", f"%[r{i}]", f"%[mh{i - 1}]", "vcc")
    p("addc", "%[top]", "vcc", "%[top]", "0", "vcc")
    # chain C: r[1..7] += H[0..6] ; top += H7 + carry (may pass 2^32 -> top2)
    p("add_co", "%[r1]", "vcc", "%[r1]", "%[t8]")
    for i in range(2, 8):
        p("addc", f"%[r{i}]", "vcc", f"%[r{i}]", f"%[t{7 + i}]", "vcc")
    p("addc", "%[top]", "vcc", "%[top]", "%[t15]", "vcc")
    p("addc", "%[top2]", "vcc", "0", "0", "vcc")
    # fold 1: value = r + T * (2^32 + 977), T = top + top2*2^32 (< 2^33):
    # T*(2^32+977) = s0 + s1*2^32 + s2*2^64 with s0:s1' = top*977 (+ top2*977
    # in s1'), s1 = s1' + top, s2 = top2 + carry -- one chain adds all three.
    p("mad", pair(0), "vcc", "%[top]", "%[k977]", "0")          # v0:v1 = top*977
    p("mul24", "v2", "0x3d1", "%[top2]")                        # top2*977 (top2 <= 1)
    p("add", "v1", "v1", "v2")                                  # < 2^11, no carry
    p("add_co", "v1", "vcc", "v1", "%[top]")                    # s1
    p("addc", "v2", "vcc", "%[top2]", "0", "vcc")               # s2 <= 2
    p("add_co", "%[r0]", "vcc", "%[r0]", "v0")
    p("addc", "%[r1]", "vcc", "%[r1]", "v1", "vcc")
    p("addc", "%[r2]", "vcc", "%[r2]", "v2", "vcc")
    for i in range(3, 8):
        p("addc", f"%[r{i}]", "vcc", f"%[r{i}]", "0", "vcc")
    p("addc", "v3", "vcc", "0", "0", "vcc")                     # carry c3 in {0,1}
    # fold 2: a wrap leaves r < 2^77; add c3*(2^32+977) into limbs 0..2
    p("mul24", "v2", "0x3d1", "v3")
    p("add_co", "%[r0]", "vcc", "%[r0]", "v2")
    p("addc", "%[r1]", "vcc", "%[r1]", "v3", "vcc")
    p("addc", "%[r2]", "vcc", "%[r2]", "0", "vcc")
    return p


def gen_add():
    p = Prog()
    p("add_co", "%[r0]", "vcc", "%[a0]", "%[b0]")
    for i in range(1, 8):
        p("addc", f"%[r{i}]", "vcc", f"%[a{i}]", f"%[b{i}]", "vcc")
    for _ in range(2):
        p("addc", "v1", "vcc", "0", "0", "vcc")                 # carry c
        p("mul24", "v0", "0x3d1", "v1")
        p("add_co", "%[r0]", "vcc", "%[r0]", "v0")
        p("addc", "%[r1]", "vcc", "%[r1]", "v1", "vcc")
        if _ == 0:
            for i in range(2, 8):
                p("addc", f"%[r{i}]", "vcc", f"%[r{i}]", "0", "vcc")
    return p


def gen_sub():
    p = Prog()
    p("sub_co", "%[r0]", "vcc", "%[a0]", "%[b0]")
    for i in range(1, 8):
        p("subb", f"%[r{i}]", "vcc", f"%[a{i}]", f"%[b{i}]", "vcc")
    for _ in range(2):
        p("addc", "v1", "vcc", "0", "0", "vcc")                 # borrow
        p("mul24", "v0", "0x3d1", "v1")
        p("sub_co", "%[r0]", "vcc", "%[r0]", "v0")
        p("subb", "%[r1]", "vcc", "%[r1]", "v1", "vcc")
        if _ == 0:
            for i in range(2, 8):
                p("subb", f"%[r{i}]", "vcc", f"%[r{i}]", "0", "vcc")
    return p


def _fold_add(p):
    """r += v1 * (2^32 + 977) (v1 small), then one more fold of the carry-out."""
    p("mul24", "v0", "0x3d1", "v1")
    p("add_co", "%[r0]", "vcc", "%[r0]", "v0")
    p("addc", "%[r1]", "vcc", "%[r1]", "v1", "vcc")
    for i in range(2, 8):
        p("addc", f"%[r{i}]", "vcc", f"%[r{i}]", "0", "vcc")
    p("addc", "v1", "vcc", "0", "0", "vcc")                     # carry-out (0/1)
    p("mul24", "v0", "0x3d1", "v1")                             # wrapped: r < 2^(s+34), no further carry
    p("add_co", "%[r0]", "vcc", "%[r0]", "v0")
    p("addc", "%[r1]", "vcc", "%[r1]", "v1", "vcc")


def gen_shl(s):
    """r = a * 2^s mod p (weak), 1 <= s <= 8: limb shifts by v_alignbit, one fold."""
    p = Prog()
    p("lshr", "v1", str(32 - s), "%[a7]")                       # bits >= 256 (< 2^s)
    for i in range(7, 0, -1):
        p("alignbit", f"%[r{i}]", f"%[a{i}]", f"%[a{i - 1}]", str(32 - s))
    p("lshl", "%[r0]", str(s), "%[a0]")
    _fold_add(p)
    return p


def gen_mul3():
    """r = 3a mod p (weak): 2a by v_alignbit, + a in one chain, one fold."""
    p = Prog()
    p("lshr", "v1", "31", "%[a7]")
    for i in range(7, 0, -1):
        p("alignbit", f"%[r{i}]", f"%[a{i}]", f"%[a{i - 1}]", "31")
    p("lshl", "%[r0]", "1", "%[a0]")
    p("add_co", "%[r0]", "vcc", "%[r0]", "%[a0]")
    for i in range(1, 8):
        p("addc", f"%[r{i}]", "vcc", f"%[r{i}]", f"%[a{i}]", "vcc")
    p("addc", "v1", "vcc", "v1", "0", "vcc")                    # bits >= 256: 0..2
    _fold_add(p)
    return p


def gen_sub_shl(s):
    """r = a - b * 2^s mod p (weak), 1 <= s <= 8.

    The low 256 bits of b<<s are formed in r and subtracted from a in one borrow
    chain; top bits and the borrow both stand for multiples of 2^256 == 2^32 + 977,
    so k = top + borrow copies of (2^32 + 977) are subtracted, and a final borrow
    is folded once more (the wrapped value is then >= 2^256 - 2^42: no further
    borrow)."""
    p = Prog()
    p("lshr", "v1", str(32 - s), "%[b7]")
    for i in range(7, 0, -1):
        p("alignbit", f"%[r{i}]", f"%[b{i}]", f"%[b{i - 1}]", str(32 - s))
    p("lshl", "%[r0]", str(s), "%[b0]")
    p("sub_co", "%[r0]", "vcc", "%[a0]", "%[r0]")
    for i in range(1, 8):
        p("subb", f"%[r{i}]", "vcc", f"%[a{i}]", f"%[r{i}]", "vcc")
    p("addc", "v0", "vcc", "v1", "0", "vcc")                    # k = top + borrow
    p("mul24", "v1", "0x3d1", "v0")
    p("sub_co", "%[r0]", "vcc", "%[r0]", "v1")
    p("subb", "%[r1]", "vcc", "%[r1]", "v0", "vcc")
    for i in range(2, 8):
        p("subb", f"%[r{i}]", "vcc", f"%[r{i}]", "0", "vcc")
    p("addc", "v0", "vcc", "0", "0", "vcc")                     # borrow-out (0/1)
    p("mul24", "v1", "0x3d1", "v0")
    p("sub_co", "%[r0]", "vcc", "%[r0]", "v1")
    p("subb", "%[r1]", "vcc", "%[r1]", "v0", "vcc")
    return p


# -------------------------------------------------------------- text output
def fmt(ins):
    op = ins[0]
    a = ins[1:]
    if op == "mad":
        return f"v_mad_u64_u32 {a[0]}, {a[1]}, {a[2]}, {a[3]}, {a[4]}"
    if op == "addc":
        return f"v_addc_co_u32 {a[0]}, {a[1]}, {a[2]}, {a[3]}, {a[4]}"
    if op == "add_co":
        return f"v_add_co_u32 {a[0]}, {a[1]}, {a[2]}, {a[3]}"
    if op == "sub_co":
        return f"v_sub_co_u32 {a[0]}, {a[1]}, {a[2]}, {a[3]}"
    if op == "subb":
        return f"v_subb_co_u32 {a[0]}, {a[1]}, {a[2]}, {a[3]}, {a[4]}"
    if op == "mov":
        return f"v_mov_b32 {a[0]}, {a[1]}"
    if op == "alignbit":
        return f"v_alignbit_b32 {a[0]}, {a[1]}, {a[2]}, {a[3]}"
    if op == "lshl1":
        return f"v_lshlrev_b32 {a[0]}, 1, {a[1]}"
    if op == "lshr31":
        return f"v_lshrrev_b32 {a[0]}, 31, {a[1]}"
    if op == "lshl":
        return f"v_lshlrev_b32 {a[0]}, {a[1]}, {a[2]}"
    if op == "lshr":
        return f"v_lshrrev_b32 {a[0]}, {a[1]}, {a[2]}"
    if op == "mul24":
        return f"v_mul_u32_u24_e32 {a[0]}, {a[1]}, {a[2]}"
    if op == "add":
        return f"v_add_u32 {a[0]}, {a[1]}, {a[2]}"
    raise ValueError(op)


def macro(name, params, prog, outs, ins, clobbers, sgpr_temps=()):
    body = "\\n\\t".join(fmt(i) for i in prog.ins)
    out_s = ", ".join(outs + [f'[{s}] "=&s"(gv_sc_tmp_)' for s in sgpr_temps])
    lines = [f"#define {name}({', '.join(params)}) \\"]
    if sgpr_temps:
        lines.append("  do { uint64_t gv_sc_tmp_; \\")
    lines.append(f'  asm volatile("{body}" \\')
    lines.append(f"    : {out_s} \\")
    lines.append(f"    : {', '.join(ins)} \\")
    lines.append(f"    : {', '.join(clobbers)})" + ("; } while (0)" if sgpr_temps else ""))
    return "\n".join(lines) + "\n"


def generate():
    parts = ["// GENERATED by tools/gen_field_asm.py -- do not edit by hand.\n"
             "// Every carry chain is back-to-back; see the generator for the rationale.\n"]
    V = ['"v0"', '"v1"', '"v2"', '"v3"', '"vcc"']
    parts.append(macro("GV_MUL512_ASM", ["T", "A", "B"], gen_mul512(),
                       [f'[t{k}] "=&v"((T)[{k}])' for k in range(16)],
                       [f'[a{i}] "v"((A)[{i}])' for i in range(8)] + [f'[b{i}] "v"((B)[{i}])' for i in range(8)],
                       V))
    parts.append(macro("GV_SQRX_ASM", ["C", "A"], gen_sqr_cross(),
                       [f'[c{k}] "=&v"((C)[{k}])' for k in range(1, 16)],
                       [f'[a{i}] "v"((A)[{i}])' for i in range(8)], V))
    parts.append(macro("GV_SQRF_ASM", ["T", "C", "SQ"], gen_sqr_finish(),
                       [f'[t{k}] "=&v"((T)[{k}])' for k in range(16)],
                       [f'[c{k}] "v"((C)[{k}])' for k in range(1, 16)] +
                       [f'[sl{i}] "v"((uint32_t)(SQ)[{i}])' for i in range(8)] +
                       [f'[sh{i}] "v"((uint32_t)((SQ)[{i}] >> 32))' for i in range(8)], ['"vcc"']))
    parts.append(macro("GV_REDUCE_ASM", ["R", "T", "M", "TOP", "TOP2"], gen_reduce(),
                       [f'[r{i}] "=&v"((R)[{i}])' for i in range(8)] + ['[top] "=&v"(TOP)', '[top2] "=&v"(TOP2)'],
                       [f'[t{i}] "v"((T)[{i}])' for i in range(16)] +
                       [f'[ml{i}] "v"((uint32_t)(M)[{i}])' for i in range(8)] +
                       [f'[mh{i}] "v"((uint32_t)((M)[{i}] >> 32))' for i in range(8)] + ['[k977] "s"(977u)'],
                       V))
    parts.append(macro("GV_ADD_ASM", ["R", "A", "B"], gen_add(),
                       [f'[r{i}] "=&v"((R)[{i}])' for i in range(8)],
                       [f'[a{i}] "v"((A)[{i}])' for i in range(8)] + [f'[b{i}] "v"((B)[{i}])' for i in range(8)],
                       ['"v0"', '"v1"', '"vcc"']))
    parts.append(macro("GV_SUB_ASM", ["R", "A", "B"], gen_sub(),
                       [f'[r{i}] "=&v"((R)[{i}])' for i in range(8)],
                       [f'[a{i}] "v"((A)[{i}])' for i in range(8)] + [f'[b{i}] "v"((B)[{i}])' for i in range(8)],
                       ['"v0"', '"v1"', '"vcc"']))
    R8 = [f'[r{i}] "=&v"((R)[{i}])' for i in range(8)]
    A8 = [f'[a{i}] "v"((A)[{i}])' for i in range(8)]
    B8 = [f'[b{i}] "v"((B)[{i}])' for i in range(8)]
    for sh in (1, 2, 3):
        parts.append(macro(f"GV_SHL{sh}_ASM", ["R", "A"], gen_shl(sh), R8, A8, ['"v0"', '"v1"', '"vcc"']))
        parts.append(macro(f"GV_SUBSHL{sh}_ASM", ["R", "A", "B"], gen_sub_shl(sh), R8, A8 + B8,
                           ['"v0"', '"v1"', '"vcc"']))
    parts.append(macro("GV_MUL3_ASM", ["R", "A"], gen_mul3(), R8, A8, ['"v0"', '"v1"', '"vcc"']))
    return "\n".join(parts)


# ----------------------------------------------------------------- emulator
class Machine:
    """Executes instruction tuples: 32-bit VGPRs, 64-bit lane-mask carries."""

    def __init__(self, env):
        self.r = dict(env)           # name -> value (u32 for v regs/operands)
        self.carry = {}              # "vcc"/sgpr name -> 0/1

    def val(self, x):
        if x == "vcc":
            return self.carry.get(x, 0)
        if x.startswith("%["):
            return self.r[x[2:-1]]
        if x.startswith("v[") or x.startswith("v"):
            if x.startswith("v["):
                lo, hi = x[2:-1].split(":")
                return self.r.get(f"v{lo}", 0) | (self.r.get(f"v{hi}", 0) << 32)
            return self.r.get(x, 0)
        if x == "vcc" or x.startswith("%[s"):
            return self.carry.get(x, 0)
        return int(x, 0)

    def setv(self, x, v):
        if x.startswith("v["):
            lo, hi = x[2:-1].split(":")
            self.r[f"v{lo}"] = v & M32
            self.r[f"v{hi}"] = (v >> 32) & M32
        elif x.startswith("%["):
            self.r[x[2:-1]] = v & M32
        else:
            self.r[x] = v & M32

    def run(self, prog):
        for ins in prog.ins:
            op, a = ins[0], ins[1:]
            if op == "mad":
                s = self.val(a[2]) * self.val(a[3]) + self.val(a[4])
                self.setv(a[0], s)
                self.carry[a[1]] = s >> 64
            elif op == "addc":
                s = self.val(a[2]) + self.val(a[3]) + self.carry.get(a[4], 0)
                self.setv(a[0], s)
                self.carry[a[1]] = s >> 32
            elif op == "add_co":
                s = self.val(a[2]) + self.val(a[3])
                self.setv(a[0], s)
                self.carry[a[1]] = s >> 32
            elif op == "sub_co":
                s = self.val(a[2]) - self.val(a[3])
                self.setv(a[0], s)
                self.carry[a[1]] = 1 if s < 0 else 0
            elif op == "subb":
                s = self.val(a[2]) - self.val(a[3]) - self.carry.get(a[4], 0)
                self.setv(a[0], s)
                self.carry[a[1]] = 1 if s < 0 else 0
            elif op == "mov":
                self.setv(a[0], self.val(a[1]))
            elif op == "alignbit":
                v = ((self.val(a[1]) << 32) | self.val(a[2])) >> self.val(a[3])
                self.setv(a[0], v)
            elif op == "lshl1":
                self.setv(a[0], self.val(a[1]) << 1)
            elif op == "lshr31":
                self.setv(a[0], self.val(a[1]) >> 31)
            elif op == "lshl":
                self.setv(a[0], self.val(a[2]) << int(a[1]))
            elif op == "lshr":
                self.setv(a[0], self.val(a[2]) >> int(a[1]))
            elif op == "mul24":
                self.setv(a[0], (self.val(a[1]) & 0xFFFFFF) * (self.val(a[2]) & 0xFFFFFF))
            elif op == "add":
                self.setv(a[0], self.val(a[1]) + self.val(a[2]))
            else:
                raise ValueError(op)
        return self


def hazard_check(prog):
    """Every instruction reading a carry must directly follow that carry's writer."""
    last_write = {}
    for idx, ins in enumerate(prog.ins):
        op, a = ins[0], ins[1:]
        reads = []
        if op in ("addc", "subb"):
            reads = [a[4]]
        for c in reads:
            w = last_write.get(c)
            if w is None or w != idx - 1:
                return f"instruction {idx} ({fmt(ins)}) reads {c} written at {w}"
        if op in ("mad", "addc", "add_co", "sub_co", "subb"):
            last_write[a[1]] = idx
    return None


def limbs(x, n):
    return [(x >> (32 * i)) & M32 for i in range(n)]


def join(vals):
    return sum(v << (32 * i) for i, v in enumerate(vals))


def emu_mul512(a, b):
    env = {f"a{i}": v for i, v in enumerate(limbs(a, 8))}
    env.update({f"b{i}": v for i, v in enumerate(limbs(b, 8))})
    m = Machine(env).run(gen_mul512())
    return join([m.r[f"t{k}"] for k in range(16)])


def emu_sqr(a):
    env = {f"a{i}": v for i, v in enumerate(limbs(a, 8))}
    m = Machine(env).run(gen_sqr_cross())
    c = {k: m.r[f"c{k}"] for k in range(1, 16)}
    env2 = {f"c{k}": c[k] for k in c}
    al = limbs(a, 8)
    for i in range(8):
        sq = al[i] * al[i]
        env2[f"sl{i}"] = sq & M32
        env2[f"sh{i}"] = sq >> 32
    m2 = Machine(env2).run(gen_sqr_finish())
    return join([m2.r[f"t{k}"] for k in range(16)])


def emu_reduce(t):
    tl = limbs(t, 16)
    env = {f"t{i}": v for i, v in enumerate(tl)}
    for i in range(8):
        mm = tl[8 + i] * 977
        env[f"ml{i}"] = mm & M32
        env[f"mh{i}"] = mm >> 32
    env["k977"] = 977
    m = Machine(env).run(gen_reduce())
    return join([m.r[f"r{i}"] for i in range(8)])


def emu_add(a, b):
    env = {f"a{i}": v for i, v in enumerate(limbs(a, 8))}
    env.update({f"b{i}": v for i, v in enumerate(limbs(b, 8))})
    m = Machine(env).run(gen_add())
    return join([m.r[f"r{i}"] for i in range(8)])


def emu_sub(a, b):
    env = {f"a{i}": v for i, v in enumerate(limbs(a, 8))}
    env.update({f"b{i}": v for i, v in enumerate(limbs(b, 8))})
    m = Machine(env).run(gen_sub())
    return join([m.r[f"r{i}"] for i in range(8)])


def emu_shl(a, sh):
    env = {f"a{i}": v for i, v in enumerate(limbs(a, 8))}
    m = Machine(env).run(gen_shl(sh))
    return join([m.r[f"r{i}"] for i in range(8)])


def emu_mul3(a):
    env = {f"a{i}": v for i, v in enumerate(limbs(a, 8))}
    m = Machine(env).run(gen_mul3())
    return join([m.r[f"r{i}"] for i in range(8)])


def emu_sub_shl(a, b, sh):
    env = {f"a{i}": v for i, v in enumerate(limbs(a, 8))}
    env.update({f"b{i}": v for i, v in enumerate(limbs(b, 8))})
    m = Machine(env).run(gen_sub_shl(sh))
    return join([m.r[f"r{i}"] for i in range(8)])


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    out = os.path.join(here, "..", "cosmos-sdk-rootchain_amd", "csrc", "secp_field_asm.inc")
    with open(out, "w") as f:
        f.write(generate())
    for name, g in (("mul512", gen_mul512), ("sqrx", gen_sqr_cross), ("sqrf", gen_sqr_finish),
                    ("reduce", gen_reduce), ("add", gen_add), ("sub", gen_sub)):
        prog = g()
        print(f"{name:7s} {len(prog.ins):4d} instructions; hazard: {hazard_check(prog)}")
    print("wrote", os.path.normpath(out))
