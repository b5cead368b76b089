// ed_lat.hip -- small ed25519 batches against cached keys:
// the IBC 07-tendermint commit checks (a validator set's keys sign every
// block) and multisig ed25519 sub-keys of accounts, on the limb-sliced field
// layer (ed_fsl.cuh).  Same verdict as go1.14 crypto/ed25519 Verify (via
// tendermint v0.33.4 PubKeyEd25519.VerifyBytes) and as the throughput
// kernels (ed_verify.hip); only the schedule differs.
//
//   k_ed_keys    one lane per key: FromBytes(A) (the reference's lenient
//                decode), then the comb table of -A: j * 16^w * (-A) for
//                w < 64, j = 1..8, cached form (Y+X, Y-X, 2Z, 2dT), no
//                inversion: 73,728 B per key; the raw key bytes (hashed by
//                Verify) and the decode verdict beside it.
//   k_ed_lat_sl  one signature per 256-thread block.  Phase 1, concurrently:
//                wave 0 stages the message in LDS and computes
//                h = SHA-512(R || A || M) mod L and its 64 signed radix-16
//                digits; wave 1 decodes R strictly (efsl_decode_strict: the
//                point R' must equal, so no inversion of Z' is needed) and
//                checks S (sig[63] & 224, ScMinimal); waves 2-3 add the 32
//                [s]B comb entries (4 per row).  Phase 2: the 16 rows add the
//                64 [h](-A) entries of the key's table (4 per row) -- no
//                doublings at all --, two shuffle rounds per wave and two more
//                in wave 0 sum the rows, and R' == (x_R, y_R) is checked
//                projectively.
//   k_ed_lat_unc small batches against UNCACHED keys (first-seen multisig
//                sub-keys, gv_verify_ed25519_msgs up to "ed_unc_lat_max"):
//                FromBytes(A) and j (-A) in the kernel, the 252-doubling
//                ladder on four waves with one point per wave spread over its
//                rows (see the kernel's comment).
#include <hip/hip_runtime.h>

#include "ed_fsl.cuh"
#include "gv_kernels.h"

#if defined(__HIP_DEVICE_COMPILE__) && defined(__AMDGCN_WAVEFRONT_SIZE) && __AMDGCN_WAVEFRONT_SIZE != 64
#error "ed_lat.hip places four 16-lane rows in a wave64"
#endif

namespace gv {
namespace ed {

static_assert(GV_EDK_WORDS == 64 * 8 * ED_CACHED_WORDS, "key table size");

__global__ __launch_bounds__(64) void k_ed_keys(const uint8_t* pub32, uint32_t n, uint32_t base, uint32_t* ktab,
                                                uint32_t* kpub, uint32_t* kok) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (g >= n) return;
  u32 pw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint8_t* p = pub32 + (size_t)g * 32 + 4 * i;
    pw[i] = (u32)p[0] | ((u32)p[1] << 8) | ((u32)p[2] << 16) | ((u32)p[3] << 24);
    kpub[(size_t)(base + g) * 8 + i] = pw[i];
  }
  ge_ext a, P;
  const bool ok = ge_frombytes(a, pw);
  kok[base + g] = ok ? 1u : 0u;
  ge_neg(P, a);
  u32* tab = ktab + (size_t)(base + g) * GV_EDK_WORDS;
#pragma unroll 1
  for (int w = 0; w < 64; ++w) {
    if (w) {
      ge_dbl_t<false>(P, P);
      ge_dbl_t<false>(P, P);
      ge_dbl_t<false>(P, P);
      ge_dbl_t<true>(P, P);
    }
    ge_cached c1, c;
    ge_to_cached(c1, P);
    atab_store(tab + (size_t)(w * 8) * ED_CACHED_WORDS, 1, 0, c1);
    ge_ext acc = P;
#pragma unroll 1
    for (int j = 2; j <= 8; ++j) {
      ge_add_cached(acc, acc, c1, false);
      ge_to_cached(c, acc);
      atab_store(tab + (size_t)(w * 8 + j - 1) * ED_CACHED_WORDS, 1, 0, c);
    }
  }
}

// The same tables in two launches, so the 448 table additions per key leave
// the serial chain: k_ed_keys_chain (lane = key) runs FromBytes and the 252
// doublings and parks the 64 window bases 16^w (-A) (extended coordinates,
// 36 words each, in scratch); k_ed_keys_tab (lane = key x window) adds each
// base to itself seven times into the table -- the same operations on the
// same values as k_ed_keys, so the same table words.
GV_DEV void ext_store(u32* p, const ge_ext& a) {
#pragma unroll
  for (int i = 0; i < 9; ++i) { p[i] = a.X.n[i]; p[9 + i] = a.Y.n[i]; p[18 + i] = a.Z.n[i]; p[27 + i] = a.T.n[i]; }
}
GV_DEV void ext_load(ge_ext& a, const u32* p) {
#pragma unroll
  for (int i = 0; i < 9; ++i) { a.X.n[i] = p[i]; a.Y.n[i] = p[9 + i]; a.Z.n[i] = p[18 + i]; a.T.n[i] = p[27 + i]; }
}
// RB: the comb's radix bits -- 4 (the key arena's tables, 64 windows of 8
// entries, read by k_ed_lat_sl too) or 6 (the grouped route's per-batch
// tables: 43 windows of 32 entries, 43 additions per [h](-A) instead of 64).
template <int RB>
struct EdComb {
  static constexpr int NW = RB == 4 ? 64 : 43;              // windows over h < 2^253
  static constexpr int NE = 1 << (RB - 1);                  // entries j = 1..NE per window
  static constexpr size_t WORDS = (size_t)NW * NE * ED_CACHED_WORDS;
};
static_assert(EdComb<4>::WORDS == GV_EDK_WORDS && EdComb<6>::WORDS == GV_EDK64_WORDS, "comb table sizes");

template <int RB>
__global__ __launch_bounds__(64) void k_ed_keys_chain(const uint8_t* pub32, uint32_t n, uint32_t base, uint32_t* kpub,
                                                      uint32_t* kok, uint32_t* wbase) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (g >= n) return;
  u32 pw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint8_t* p = pub32 + (size_t)g * 32 + 4 * i;
    pw[i] = (u32)p[0] | ((u32)p[1] << 8) | ((u32)p[2] << 16) | ((u32)p[3] << 24);
    kpub[(size_t)(base + g) * 8 + i] = pw[i];
  }
  ge_ext a, P;
  const bool ok = ge_frombytes(a, pw);
  kok[base + g] = ok ? 1u : 0u;
  ge_neg(P, a);
  using L = EdComb<RB>;
  u32* wb = wbase + (size_t)g * L::NW * ED_CACHED_WORDS;
#pragma unroll 1
  for (int w = 0; w < L::NW; ++w) {
    if (w) {
#pragma unroll 1
      for (int k = 0; k < RB - 1; ++k) ge_dbl_t<false>(P, P);
      ge_dbl_t<true>(P, P);
    }
    ext_store(wb + (size_t)w * ED_CACHED_WORDS, P);
  }
}
template <int RB>
__global__ __launch_bounds__(256) void k_ed_keys_tab(uint32_t n, uint32_t base, uint32_t* ktab, const uint32_t* wbase) {
  using L = EdComb<RB>;
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n * (uint32_t)L::NW) return;
  const uint32_t g = t / (uint32_t)L::NW, w = t % (uint32_t)L::NW;
  ge_ext P;
  ext_load(P, wbase + (size_t)t * ED_CACHED_WORDS);
  u32* tab = ktab + (size_t)(base + g) * L::WORDS;
  ge_cached c1, c;
  ge_to_cached(c1, P);
  atab_store(tab + (size_t)(w * L::NE) * ED_CACHED_WORDS, 1, 0, c1);
  ge_ext acc = P;
#pragma unroll 1
  for (int j = 2; j <= L::NE; ++j) {
    ge_add_cached(acc, acc, c1, false);
    ge_to_cached(c, acc);
    atab_store(tab + (size_t)(w * L::NE + j - 1) * ED_CACHED_WORDS, 1, 0, c);
  }
}

#define EDL_MSG_LDS 2048                    // padded SHA-512 inputs up to 16 blocks take the LDS path
// GV_EDL_SHA_VALU: the LDS-path SHA-512 on the VALU with the schedules of all
// blocks expanded at once (sha512_wave); 0: the scalar-unit compression.
#ifndef GV_EDL_SHA_VALU
#define GV_EDL_SHA_VALU 1
#endif

struct EdlShared {
  union {                                   // the padded SHA-512 input (wave 0): R || A || M || padding
    u32 pre[16];
    uint8_t msg[EDL_MSG_LDS];
    uint64_t words[EDL_MSG_LDS / 8];
  };
  uint64_t wk[EDL_MSG_LDS / 128][80];       // each block's message schedule + round constants (sha512_wave)
  int hd[64];                               // signed radix-16 digits of h
  u32 xr[16], yr[16];                       // the decoded R, sliced
  u32 flags;                                // bit 0: R decodes, bit 1: S checks
  u32 pt[4][4][16];                         // wave sums X, Y, Z, T
};

// SHA-512 of the nblocks blocks staged in sh.words (one wave, every lane
// alike), on the VALU.  Lane b < nblocks expands block b's message schedule
// into sh.wk (W_t + K_t), all blocks at once; then the 80 rounds of each
// block run with the state in VGPRs: a lane-varying zero added to the state
// keeps the compiler from moving the (uniform) chain to the scalar unit,
// where a 64-bit rotate is three dependent SALU operations -- on the VALU it
// is two v_alignbit, and the xor / choose / majority terms fold into
// three-input v_xor3 / v_bitop3.
GV_DEV uint64_t sha_rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
// 64-bit values as (lo, hi) 32-bit halves: a rotate is two v_alignbit, the
// three-term xors one v_xor3 per half
struct u64p { u32 lo, hi; };
template <int N>
GV_DEV u64p rotr_p(u64p x) {
  if constexpr (N < 32) return {__builtin_amdgcn_alignbit(x.hi, x.lo, N), __builtin_amdgcn_alignbit(x.lo, x.hi, N)};
  else return {__builtin_amdgcn_alignbit(x.lo, x.hi, N - 32), __builtin_amdgcn_alignbit(x.hi, x.lo, N - 32)};
}
// gfx950 v_bitop3_b32: any function of three inputs (truth table indexed by
// a*4 + b*2 + c): 0x96 a ^ b ^ c, 0xCA choose (a ? b : c), 0xE8 majority
template <int TT>
GV_DEV u64p bop3_p(u64p a, u64p b, u64p c) {
  return {(u32)__builtin_amdgcn_bitop3_b32(a.lo, b.lo, c.lo, TT), (u32)__builtin_amdgcn_bitop3_b32(a.hi, b.hi, c.hi, TT)};
}
GV_DEV u64p xor3_p(u64p a, u64p b, u64p c) { return bop3_p<0x96>(a, b, c); }
GV_DEV u64p to_p(uint64_t v) { return {(u32)v, (u32)(v >> 32)}; }
GV_DEV uint64_t from_p(u64p v) { return ((uint64_t)v.hi << 32) | v.lo; }
template <class SH>
GV_DEV void sha512_wave(uint64_t hs[8], SH& sh, u32 nblocks, u32 lane) {
  if (lane < nblocks) {
    uint64_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      w[j] = __builtin_bswap64(sh.words[lane * 16u + (u32)j]);
      sh.wk[lane][j] = w[j] + kSha512K[j];
    }
#pragma unroll
    for (int t = 16; t < 80; ++t) {
      const u64p w15 = to_p(w[(t - 15) & 15]), w2 = to_p(w[(t - 2) & 15]);
      const uint64_t s0 = from_p(xor3_p(rotr_p<1>(w15), rotr_p<8>(w15), to_p(w[(t - 15) & 15] >> 7)));
      const uint64_t s1 = from_p(xor3_p(rotr_p<19>(w2), rotr_p<61>(w2), to_p(w[(t - 2) & 15] >> 6)));
      w[t & 15] += s0 + w[(t - 7) & 15] + s1;
      sh.wk[lane][t] = w[t & 15] + kSha512K[t];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  u32 vz;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
  uint64_t st[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) st[i] = hs[i] + vz;
#pragma unroll 1
  for (u32 blk = 0; blk < nblocks; ++blk) {
    uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], hh = st[7];
#pragma unroll
    for (int t = 0; t < 80; ++t) {
      const u64p ep = to_p(e), ap = to_p(a);
      const uint64_t S1 = from_p(xor3_p(rotr_p<14>(ep), rotr_p<18>(ep), rotr_p<41>(ep)));
      const uint64_t ch = from_p(bop3_p<0xCA>(ep, to_p(f), to_p(g)));      // (e & f) ^ (~e & g)
      const uint64_t t1 = hh + S1 + ch + sh.wk[blk][t];
      const uint64_t S0 = from_p(xor3_p(rotr_p<28>(ap), rotr_p<34>(ap), rotr_p<39>(ap)));
      const uint64_t mj = from_p(bop3_p<0xE8>(ap, to_p(b), to_p(c)));     // majority
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += hh;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) hs[i] = st[i];
}

// Wave-wide: h = SHA-512(R || A || M) mod L and its 64 signed radix-16 digits
// into sh.hd; sw = the signature words, aw = A's words (the bytes Verify hashes).
template <class SH>
GV_DEV void edl_hash_digits(SH& sh, const u32 sw[16], const u32 aw[8], const uint8_t* m, u32 len, u32 lane) {
  // the message staged in LDS first (one load per lane per 64 bytes instead
  // of a serial byte stream)
  const u32 total = 64u + len, nblocks = (total + 17u + 127u) >> 7, padded = nblocks << 7;
  u32 dig[16], h[8];
  if (padded <= EDL_MSG_LDS) {
    // the whole SHA-512 input -- R || A || M, 0x80, zeros, the 128-bit
    // big-endian bit length -- laid out in LDS by the wave (one load per
    // lane per 64 message bytes); the compression then reads each block's
    // sixteen 64-bit words with uniform addresses and runs on the scalar unit
    if (lane < 8u) sh.pre[lane] = sw[lane];
    else if (lane < 16u) sh.pre[lane] = aw[lane - 8u];
    const uint64_t bits = (uint64_t)total * 8u;
    for (u32 i = 64u + lane; i < padded; i += 64u) {
      u32 byte = 0;
      if (i < total) byte = m[i - 64u];
      else if (i == total) byte = 0x80u;
      else if (i >= padded - 8u) byte = (u32)(bits >> (8u * (padded - 1u - i))) & 0xFFu;
      sh.msg[i] = (uint8_t)byte;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    uint64_t hs[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull, 0xa54ff53a5f1d36f1ull,
                      0x510e527fade682d1ull, 0x9b05688c2b3e6c1full, 0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
#if GV_EDL_SHA_VALU
    sha512_wave(hs, sh, nblocks, lane);
#else
#pragma unroll 1
    for (u32 blk = 0; blk < nblocks; ++blk) {
      uint64_t w[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = __builtin_bswap64(sh.words[blk * 16u + (u32)j]);
      sha512_compress(hs, w);
    }
#endif
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      dig[2 * i] = __builtin_bswap32((u32)(hs[i] >> 32));
      dig[2 * i + 1] = __builtin_bswap32((u32)hs[i]);
    }
  } else {                                            // long messages: byte stream from memory
    u32 pre[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      pre[i] = sw[i];
      pre[8 + i] = aw[i];
    }
    sha512_pre64(dig, pre, [=](u32 i) { return (u32)m[i]; }, len);
  }
  sc_reduce512(h, dig);
  const uint64_t car = sc_radix16_carries(h);
  const u32 nib = (h[lane >> 3] >> (4u * (lane & 7u))) & 15u;
  const int cin = lane > 0u ? (int)((car >> (lane - 1u)) & 1u) : 0;
  const int cout = lane < 63u ? (int)((car >> lane) & 1u) : 0;
  sh.hd[lane] = (int)nib + cin - 16 * cout;
}

__global__ __launch_bounds__(256) void k_ed_lat_sl(const gvk_edl b) {
  __shared__ EdlShared sh;
  const u32 gi = blockIdx.x;                // grid = n: every block is live
  const u32 lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  u32 sl = b.slot[gi];
  bool kok = sl < b.kcount;
  if (!kok) sl = 0;                         // the arena always holds slot 0's memory
  kok = kok && b.kok[sl] != 0u;
  u32 sw[16];
  {
    const uint4* sp = (const uint4*)(b.sig64 + (size_t)gi * 64);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = sp[q];
      sw[4 * q] = v.x; sw[4 * q + 1] = v.y; sw[4 * q + 2] = v.z; sw[4 * q + 3] = v.w;
    }
  }
  const fslk k = efsl_consts();
  const u32 L = k.L, row = threadIdx.x >> 4;            // row 0..15
  const bool lo = L < 9u;
  gesl A;
  gesl_identity(A, k);
  if (wave == 0u) {
    u32 aw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) aw[i] = b.kpub[(size_t)sl * 8 + i];
    edl_hash_digits(sh, sw, aw, b.msg_blob ? b.msg_blob + b.msg_off[gi] : nullptr, b.msg_len[gi], lane);
  } else if (wave == 1u) {
    u32 x, y;
    const bool rok = efsl_decode_strict(x, y, sw, k);
    const bool sok = (sw[15] >> 29) == 0u && sc_minimal(sw + 8);   // sig[63] & 224 == 0, ScMinimal
    if (lane < 16u) {
      sh.xr[L] = x;
      sh.yr[L] = y;
    }
    if (lane == 0u) sh.flags = (rok ? 1u : 0u) | (sok ? 2u : 0u);
  } else {
    // [s]B: signed radix-256 digits of s (LSB-first carries, ed_ladder_check's
    // recoding), windows r, r+8, r+16, r+24 of this row of waves 2-3
    u32 cmask = 0, c = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const u32 byte = (sw[8 + (i >> 2)] >> (8 * (i & 3))) & 0xFFu;
      c = (byte + c) > 128u ? 1u : 0u;
      cmask |= c << i;
    }
    const u32 r8 = row - 8u;
#pragma unroll 1
    for (u32 w = r8; w < 32u; w += 8u) {
      const int byte = (int)((sw[8 + (w >> 2)] >> (8 * (w & 3))) & 0xFFu);
      const int cin = w > 0u ? (int)((cmask >> (w - 1u)) & 1u) : 0;
      const int dg = byte + cin - 256 * (int)((cmask >> w) & 1u);
      if (dg != 0) {
        const u32 mag = (u32)(dg < 0 ? -dg : dg);
        const u32* e = b.btab + (size_t)(w * ED_BTAB_ENTRIES + mag) * ED_PRE_WORDS;
        gesl_add_pre(A, A, lo ? e[L] : 0u, lo ? e[9 + L] : 0u, lo ? e[18 + L] : 0u, dg < 0, k);
      }
    }
  }
  __syncthreads();
  // [h](-A): windows row, row + 16, row + 32, row + 48 from the key's table
  const u32* kt = b.ktab + (size_t)sl * GV_EDK_WORDS;
#pragma unroll 1
  for (u32 w = row; w < 64u; w += 16u) {
    const int dg = sh.hd[w];
    if (dg != 0) {
      const u32 mag = (u32)(dg < 0 ? -dg : dg);
      const u32* e = kt + (size_t)(w * 8u + mag - 1u) * ED_CACHED_WORDS;
      gesl_add_cached(A, A, lo ? e[L] : 0u, lo ? e[9 + L] : 0u, lo ? e[18 + L] : 0u, lo ? e[27 + L] : 0u, dg < 0, k);
    }
  }
  const u32 d2 = efsl_const(kEd2D, k);
#pragma unroll 1
  for (int msk = 16; msk < 64; msk <<= 1) {
    const gesl O = gesl_shfl_xor(A, msk);
    gesl_add(A, A, O, d2, k);
  }
  if (lane < 16u && lo) {
    sh.pt[wave][0][L] = A.X; sh.pt[wave][1][L] = A.Y; sh.pt[wave][2][L] = A.Z; sh.pt[wave][3][L] = A.T;
  }
  __syncthreads();
  if (wave != 0u) return;
  const u32 part = lane >> 4;                           // wave 0, row r: wave r's sum
  A.X = lo ? sh.pt[part][0][L] : 0u;
  A.Y = lo ? sh.pt[part][1][L] : 0u;
  A.Z = lo ? sh.pt[part][2][L] : 0u;
  A.T = lo ? sh.pt[part][3][L] : 0u;
#pragma unroll 1
  for (int msk = 16; msk < 64; msk <<= 1) {
    const gesl O = gesl_shfl_xor(A, msk);
    gesl_add(A, A, O, d2, k);
  }
  // R' == (x_R, y_R): X' == x_R Z', Y' == y_R Z'
  const u32 xr = lo ? sh.xr[L] : 0u, yr = lo ? sh.yr[L] : 0u;
  u32 w1[8], w2[8], w3[8], w4[8];
  efsl_to_words(w1, A.X);
  efsl_to_words(w2, fsl_mul(xr, A.Z, k));
  efsl_to_words(w3, A.Y);
  efsl_to_words(w4, fsl_mul(yr, A.Z, k));
  u32 diff = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) diff |= (w1[i] ^ w2[i]) | (w3[i] ^ w4[i]);
  const bool ok = kok && (sh.flags & 3u) == 3u && diff == 0u;
  if (threadIdx.x == 0) b.out8[gi] = ok ? 1u : 0u;
}

// ---------------------------------------------------------------------------
// Small batches against UNCACHED keys (k_ed_lat_unc): one signature per
// 256-thread block, FromBytes(A) in the kernel, and every wave keeps ONE
// point in its four 16-lane rows with each row computing a different product
// of the same round (rows_all, secp_fsl.cuh): an a = -1 doubling is two
// rounds of four products (X^2, Y^2, Z^2, (X+Y)^2, then E F, G H, E H, F G),
// an addition of a cached point two rounds as well.
//   wave 0: h = SHA-512(R || A || M) mod L, its radix-16 digits -> ladder
//           windows 4j
//   wave 1: FromBytes(A) (the reference's lenient decode) -> j (-A), j = 1..8,
//           cached form, into LDS -> ladder windows 4j + 1
//   wave 2: R decoded strictly, S checked -> ladder windows 4j + 2
//   wave 3: [s]B (the 32 comb entries of the resident table, fetched at once)
//           -> ladder windows 4j + 3
// Each ladder wave runs the doublings of all 64 windows (from its first
// non-zero digit) and adds only its own; wave 0 sums the four partial sums and
// [s]B and compares R' with R projectively.  The same operations' results as
// ed_verify_core's (the formulas are complete), so the same verdict.

// P = 2P (dbl-2008-hwcd, a = -1): A = X^2, B = Y^2, C = 2 Z^2, E = (X+Y)^2 -
// A - B, G = B - A, F = G - C, H = -A - B; X3 = E F, Y3 = G H, T3 = E H, Z3 = F G.
GV_DEV void ge4_double(gesl& P, u32 row, const fslk& k) {
  const u32 s = rsel(row, P.X, P.Y, P.Z, P.X + P.Y);
  const rows4 p1 = rows_all(fsl_sqr(s, k));
  const u32 a = p1.r[0], bb = p1.r[1], cz = p1.r[2], sq = p1.r[3];
  // E, G < 2^31.1 / 2^30.6 stay raw; F, H are carried so every product of
  // round 2 is (raw x N-form): max_limb products < 2^60.2
  const u32 e = sq + 2u * k.bias - a - bb;
  const u32 g = bb + k.bias - a;
  const u32 h = fsl_norm(2u * k.bias - a - bb, k);
  const u32 f = fsl_norm(bb + 3u * k.bias - a - (cz << 1), k);     // < 2^31.9 before the carry pass
  const rows4 p2 = rows_all(fsl_mul(rsel(row, e, g, e, g), rsel(row, f, h, h, f), k));
  P.X = p2.r[0]; P.Y = p2.r[1]; P.T = p2.r[2]; P.Z = p2.r[3];
}

// P = P + (neg ? -q : q), q cached (Y+X, Y-X, 2Z, 2dT): gesl_add_cached's
// products in two rounds -- (Y1+X1) qa, (Y1-X1) qb, 2dT2 T1, Z1 2Z2, then
// X = (A-B)(D-C), Y = (A+B)(D+C), Z = (D+C)(D-C), T = (A-B)(A+B) (C, D
// swapped for -q).  d2z: 2 Z2, or null for an affine precomputed q
// (y+x, y-x, 2dxy): D = 2 Z1.
GV_DEV void ge4_add_cached(gesl& P, u32 ypx, u32 ymx, u32 z2, u32 t2d, bool pre, bool neg, u32 row, const fslk& k) {
  const u32 qa = neg ? ymx : ypx, qb = neg ? ypx : ymx;
  const rows4 p1 = rows_all(fsl_mul(rsel(row, P.Y + P.X, P.Y + k.bias - P.X, t2d, P.Z), rsel(row, qa, qb, P.T, z2), k));
  const u32 a = p1.r[0], b = p1.r[1], c = p1.r[2], d = pre ? P.Z << 1 : p1.r[3];
  const u32 x1 = fsl_norm(a + k.bias - b, k);
  const u32 y1 = a + b;
  const u32 dpc = d + c;
  const u32 dmc = fsl_norm(d + k.bias - c, k);
  const u32 z1 = neg ? dmc : dpc, t1 = neg ? dpc : dmc;
  const rows4 p2 = rows_all(fsl_mul(rsel(row, x1, y1, z1, x1), rsel(row, t1, z1, t1, y1), k));
  P.X = p2.r[0]; P.Y = p2.r[1]; P.Z = p2.r[2]; P.T = p2.r[3];
}

// P = P + Q, both extended
GV_DEV void ge4_add(gesl& P, const gesl& Q, u32 d2, u32 row, const fslk& k) {
  ge4_add_cached(P, Q.Y + Q.X, fsl_norm(Q.Y + k.bias - Q.X, k), Q.Z << 1, fsl_mul(Q.T, d2, k), false, false, row, k);
}

// ExtendedGroupElement.FromBytes (ge_frombytes: y = bytes mod 2^255, no
// canonicality check, x from the (p-5)/8 power, sign fix-up), sliced.
GV_DEV bool efsl_decode_lenient(u32& x, u32& y, const u32 w[8], const fslk& k) {
  y = efsl_from_words(w, k);
  const u32 one = efsl_small(1u, k);
  const u32 yy = fsl_sqr(y, k);
  const u32 u = fsl_norm(yy + k.bias - one, k);                 // y^2 - 1
  const u32 v = fsl_norm(fsl_mul(yy, efsl_const(kEdD, k), k) + one, k);   // d y^2 + 1
  const u32 v3 = fsl_mul(fsl_sqr(v, k), v, k);
  u32 t = fsl_mul(fsl_sqr(v3, k), v, k);                        // v^7
  t = efsl_pow22523(fsl_mul(t, u, k), k);                       // (u v^7)^((p-5)/8)
  x = fsl_mul(fsl_mul(t, v3, k), u, k);                         // u v^3 (u v^7)^((p-5)/8)
  const u32 vxx = fsl_mul(fsl_sqr(x, k), v, k);
  const bool root = efsl_is_zero(vxx + k.bias - u);
  const bool neg_root = efsl_is_zero(vxx + u);
  if (!root) x = fsl_mul(x, efsl_const(kEdSqrtM1, k), k);
  u32 xw[8];
  efsl_to_words(xw, x);
  if ((xw[0] & 1u) != (w[7] >> 31)) x = fsl_norm(k.bias - x, k);
  return root || neg_root;
}

// GV_LAT_TRACE (A/B builds only): per block, wall-clock stamps (100 MHz) of
// k_ed_lat_unc's phases, read back with gv_debug_edl_trace.  Off in the
// product build.
#ifndef GV_LAT_TRACE
#define GV_LAT_TRACE 0
#endif
#if GV_LAT_TRACE
__device__ uint64_t g_edl_trace[256][8];
#define EDL_STAMP(k) do { if ((threadIdx.x & 63u) == 0 && blockIdx.x < 256) g_edl_trace[blockIdx.x][k] = wall_clock64(); } while (0)
#else
#define EDL_STAMP(k) do { } while (0)
#endif

GV_DEV void edl_wave_sync() {                 // one wave's LDS writes -> the wave's other lanes
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct EduShared {
  union {                                   // the padded SHA-512 input (wave 0)
    u32 pre[16];
    uint8_t msg[EDL_MSG_LDS];
    uint64_t words[EDL_MSG_LDS / 8];
  };
  uint64_t wk[EDL_MSG_LDS / 128][80];       // each block's message schedule + round constants (sha512_wave)
  int hd[64];                               // signed radix-16 digits of h
  u32 xr[16], yr[16];                       // the decoded R, sliced
  u32 flags;                                // bit 0: R decodes, bit 1: S checks
  u32 aok;                                  // A decodes
  u32 atab[8][4][9];                        // j (-A), j = 1..8: Y+X, Y-X, 2Z, 2dT
  u32 pt[4][4][16];                         // ladder sums of waves 1..3, [s]B
  u32 bent[32][3][9];                       // the [s]B comb entries (wave 3)
  int sdg[32];                              // their signed radix-256 digits of s
  u32 flag_h, flag_a;
};

__global__ __launch_bounds__(256) void k_ed_lat_unc(const gvk_edl b) {
  __shared__ EduShared sh;
  const u32 gi = blockIdx.x;                // grid = n: every block is live
  const u32 lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const fslk k = efsl_consts();
  const u32 L = k.L, row = (threadIdx.x >> 4) & 3u;
  const bool lo = L < 9u;
  if (threadIdx.x == 0) { sh.flag_h = 0u; sh.flag_a = 0u; }
  __syncthreads();
  if (wave == 0u) EDL_STAMP(0);
  u32 sw[16], aw[8];
  {
    const uint4* sp = (const uint4*)(b.sig64 + (size_t)gi * 64);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = sp[q];
      sw[4 * q] = v.x; sw[4 * q + 1] = v.y; sw[4 * q + 2] = v.z; sw[4 * q + 3] = v.w;
    }
    const uint8_t* pa = b.pub32 + (size_t)gi * 32;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      aw[i] = (u32)pa[4 * i] | ((u32)pa[4 * i + 1] << 8) | ((u32)pa[4 * i + 2] << 16) | ((u32)pa[4 * i + 3] << 24);
  }
  const u32 d2 = efsl_const(kEd2D, k);
  gesl P;
  gesl_identity(P, k);
  if (wave == 0u) {
    edl_hash_digits(sh, sw, aw, b.msg_blob ? b.msg_blob + b.msg_off[gi] : nullptr, b.msg_len[gi], lane);
    EDL_STAMP(1);
    lds_flag_set(&sh.flag_h);
  } else if (wave == 1u) {
    u32 x, y;
    const bool aok = efsl_decode_lenient(x, y, aw, k);
    EDL_STAMP(2);
    // -A = (-x, y, 1, -x y), then j (-A) in cached form
    gesl A1;
    A1.X = fsl_norm(k.bias - x, k);
    A1.Y = y;
    A1.Z = efsl_small(1u, k);
    A1.T = fsl_mul(A1.X, y, k);
    const u32 ypx1 = A1.Y + A1.X, ymx1 = fsl_norm(A1.Y + k.bias - A1.X, k), z21 = A1.Z << 1, t2d1 = fsl_mul(A1.T, d2, k);
    gesl Q = A1;
#pragma unroll 1
    for (int j = 1; j <= 8; ++j) {
      if (j == 2) ge4_double(Q, row, k);
      else if (j > 2) ge4_add_cached(Q, ypx1, ymx1, z21, t2d1, false, false, row, k);
      const u32 t2d = j == 1 ? t2d1 : fsl_mul(Q.T, d2, k);
      const u32 ymx = fsl_norm(Q.Y + k.bias - Q.X, k);        // row-wide (DPP) before the store branch
      if (row == 0u && lo) {
        sh.atab[j - 1][0][L] = Q.Y + Q.X;
        sh.atab[j - 1][1][L] = ymx;
        sh.atab[j - 1][2][L] = Q.Z << 1;
        sh.atab[j - 1][3][L] = t2d;
      }
    }
    if (threadIdx.x == 64u) sh.aok = aok ? 1u : 0u;
    EDL_STAMP(3);
    lds_flag_set(&sh.flag_a);
  } else if (wave == 2u) {
    u32 x, y;
    const bool rok = efsl_decode_strict(x, y, sw, k);
    const bool sok = (sw[15] >> 29) == 0u && sc_minimal(sw + 8);   // sig[63] & 224 == 0, ScMinimal
    if (lane < 16u) {
      sh.xr[L] = x;
      sh.yr[L] = y;
    }
    if (lane == 0u) sh.flags = (rok ? 1u : 0u) | (sok ? 2u : 0u);
    EDL_STAMP(4);
  } else {
    // [s]B: signed radix-256 digits of s (ed_ladder_check's recoding), the
    // comb entries of windows 0..31 -- no doublings; every entry's loads in
    // flight at once (row r fetches windows r, r + 4, ...), parked in LDS
    u32 cmask = 0, c = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const u32 byte = (sw[8 + (i >> 2)] >> (8 * (i & 3))) & 0xFFu;
      c = (byte + c) > 128u ? 1u : 0u;
      cmask |= c << i;
    }
#pragma unroll
    for (int w = 0; w < 32; ++w) {
      const int byte = (int)((sw[8 + (w >> 2)] >> (8 * (w & 3))) & 0xFFu);
      const int cin = w > 0 ? (int)((cmask >> (w - 1)) & 1u) : 0;
      if (lane == (u32)w) sh.sdg[w] = byte + cin - 256 * (int)((cmask >> w) & 1u);
    }
    edl_wave_sync();
#pragma unroll
    for (u32 i = 0; i < 8u; ++i) {
      const u32 w = 4u * i + row;
      const int dg = sh.sdg[w];
      const u32 mag = (u32)(dg < 0 ? -dg : dg);
      const u32* e = b.btab + (size_t)(w * ED_BTAB_ENTRIES + mag) * ED_PRE_WORDS;
      if (lo) { sh.bent[w][0][L] = e[L]; sh.bent[w][1][L] = e[9 + L]; sh.bent[w][2][L] = e[18 + L]; }
    }
    edl_wave_sync();
#pragma unroll 1
    for (u32 w = 0; w < 32u; ++w) {
      const int dg = sh.sdg[w];
      if (dg != 0)
        ge4_add_cached(P, lo ? sh.bent[w][0][L] : 0u, lo ? sh.bent[w][1][L] : 0u, 0u, lo ? sh.bent[w][2][L] : 0u,
                       true, dg < 0, row, k);
    }
    if (row == 0u && lo) { sh.pt[3][0][L] = P.X; sh.pt[3][1][L] = P.Y; sh.pt[3][2][L] = P.Z; sh.pt[3][3][L] = P.T; }
    gesl_identity(P, k);
    EDL_STAMP(5);
  }
  lds_flag_wait(&sh.flag_h);
  lds_flag_wait(&sh.flag_a);
  // [h](-A): this wave's windows 4j + wave, MSB first
  {
    bool id = true;
#pragma unroll 1
    for (int w = 63; w >= 0; --w) {
      if (!id) {
#pragma unroll 1
        for (int dd = 0; dd < 4; ++dd) ge4_double(P, row, k);
      }
      if ((u32)(w & 3) != wave) continue;
      const int dg = sh.hd[w];
      if (dg == 0) continue;
      const u32 m = (u32)(dg < 0 ? -dg : dg) - 1u;
      ge4_add_cached(P, lo ? sh.atab[m][0][L] : 0u, lo ? sh.atab[m][1][L] : 0u, lo ? sh.atab[m][2][L] : 0u,
                     lo ? sh.atab[m][3][L] : 0u, false, dg < 0, row, k);
      id = false;
    }
  }
  if (wave == 0u) EDL_STAMP(6);
  if (wave != 0u && row == 0u && lo) {
    sh.pt[wave - 1][0][L] = P.X; sh.pt[wave - 1][1][L] = P.Y; sh.pt[wave - 1][2][L] = P.Z; sh.pt[wave - 1][3][L] = P.T;
  }
  __syncthreads();
  if (wave != 0u) return;
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    gesl O;
    O.X = lo ? sh.pt[j][0][L] : 0u; O.Y = lo ? sh.pt[j][1][L] : 0u;
    O.Z = lo ? sh.pt[j][2][L] : 0u; O.T = lo ? sh.pt[j][3][L] : 0u;
    ge4_add(P, O, d2, row, k);
  }
  // R' == (x_R, y_R): X' == x_R Z', Y' == y_R Z'
  const u32 xr = lo ? sh.xr[L] : 0u, yr = lo ? sh.yr[L] : 0u;
  u32 w1[8], w2[8], w3[8], w4[8];
  efsl_to_words(w1, P.X);
  efsl_to_words(w2, fsl_mul(xr, P.Z, k));
  efsl_to_words(w3, P.Y);
  efsl_to_words(w4, fsl_mul(yr, P.Z, k));
  u32 diff = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) diff |= (w1[i] ^ w2[i]) | (w3[i] ^ w4[i]);
  const bool ok = sh.aok != 0u && (sh.flags & 3u) == 3u && diff == 0u;
  if (threadIdx.x == 0) b.out8[gi] = ok ? 1u : 0u;
  EDL_STAMP(7);
}

// Large batches against cached keys (k_ed_keyed, one signature per lane):
// the key's comb table of -A replaces FromBytes(A), the per-lane table and
// the 252 doublings of the throughput ladder -- [h](-A) is 64 table adds, no
// doubling --, then the 32 [s]B comb adds and the encode / compare of
// ed_ladder_check.  Lanes run in slot order (perm from gv_sort.hip's counting
// sort): a validator set's commits name their keys in the same order every
// block, so item order would put 64 different 73 KB tables under one wave.
template <int RB>
__global__ __launch_bounds__(256) void k_ed_keyed(const gvk_edk b) {
  using L = EdComb<RB>;
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;
  if (g >= b.n) return;
  const uint32_t it = b.perm ? b.perm[g] : g;
  u32 sl = b.slot[it];
  bool ok = sl < b.kcount;
  if (!ok) sl = 0;                          // the arena always holds slot 0's memory
  ok = ok && b.kok[sl] != 0u;
  u32 sw[16], pre[16];
  const uint4* sp = (const uint4*)(b.sig64 + (size_t)it * 64);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint4 v = sp[q];
    sw[4 * q] = v.x; sw[4 * q + 1] = v.y; sw[4 * q + 2] = v.z; sw[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    pre[i] = sw[i];                         // R
    pre[8 + i] = b.kpub[(size_t)sl * 8 + i];   // A (the bytes Verify hashes)
  }
  const uint8_t* m = b.msg_blob ? b.msg_blob + b.msg_off[it] : nullptr;
  u32 dig[16], h[8];
  sha512_pre64(dig, pre, [=](u32 i) { return (u32)m[i]; }, b.msg_len[it]);
  sc_reduce512(h, dig);                     // ScReduce
  ok = ok && (sw[15] >> 29) == 0 && sc_minimal(sw + 8);   // sig[63] & 224 == 0, ScMinimal
  // [h](-A) = sum_w digit_w * 2^(RB w) (-A): one cached-table add per nonzero
  // signed digit in [-2^(RB-1), 2^(RB-1)), LSB-first (no doublings: any order)
  const u32* kt = b.ktab + (size_t)sl * L::WORDS;
  ge_ext acc;
  ge_identity(acc);
  int cin = 0;
#pragma unroll 1
  for (int w = 0; w < L::NW; ++w) {
    const int pos = RB * w, wi = pos >> 5;
    const uint64_t pair = (uint64_t)h[wi] | (wi < 7 ? (uint64_t)h[wi + 1] << 32 : 0ull);
    int dg = (int)((pair >> (pos & 31)) & (uint64_t)((1u << RB) - 1u)) + cin;
    cin = 0;
    if (w < L::NW - 1 && dg >= L::NE) { dg -= 1 << RB; cin = 1; }   // h < 2^253: no carry out of the top window
    if (dg != 0) {
      const int mag = dg < 0 ? -dg : dg;
      ge_add_tab<true>(acc, acc, kt + (size_t)(w * L::NE + mag - 1) * ED_CACHED_WORDS, 1, 0, dg < 0);
    }
  }
  // + [s]B: 16 signed radix-2^16 digits from btab16, or (null) 32 radix-256
  // digits, LSB-first (ed_ladder_check's recoding)
  if (b.btab16) {
    ed_add_sb16(acc, sw + 8, b.btab16);
  } else {
    u32 ss[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) ss[i] = sw[8 + i];
    int carry = 0;
#pragma unroll 1
    for (int w = 0; w < ED_BTAB_WINDOWS; ++w) {
      int dgt = (int)(ss[0] & 0xFFu) + carry;
#pragma unroll
      for (int k = 0; k < 7; ++k) ss[k] = (ss[k] >> 8) | (ss[k + 1] << 24);
      ss[7] >>= 8;
      carry = dgt > 128 ? 1 : 0;
      dgt -= 256 * carry;
      const int mag = dgt < 0 ? -dgt : dgt;
      ge_add_pretab(acc, acc, b.btab + (size_t)(w * ED_BTAB_ENTRIES + mag) * ED_PRE_WORDS, dgt < 0);
    }
  }
  u32 ew[8];
  ge_tobytes(ew, acc);
  u32 diff = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) diff |= ew[i] ^ sw[i];
  b.out8[it] = (ok && diff == 0u) ? 1u : 0u;
}

// In-batch key grouping for the throughput entry points (a relayer's batch
// of commits repeats a validator set's keys): the 32 key bytes of every item
// go into an open-addressing table (2n+ slots, atomicCAS; the first item of a
// key is its representative), representatives take dense ids (one atomic per
// wave) and copy their bytes to the compact key rows k_ed_keys reads, every
// item gets its key's id.  The verdicts are the per-item ones: the key table
// is a pure function of the 32 bytes.
GV_DEV void ed_key_words(u32 w[8], const uint8_t* pub32, u32 i) {
  const uint4* p = (const uint4*)(pub32 + (size_t)i * 32);
  const uint4 a = p[0], c = p[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = c.x; w[5] = c.y; w[6] = c.z; w[7] = c.w;
}
__global__ __launch_bounds__(256) void k_ed_dedupe(u32 n, const uint8_t* pub32, u32* table, u32 tmask, u32* rep) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  u32 w[8];
  ed_key_words(w, pub32, g);
  uint64_t h = 0x9E3779B97F4A7C15ull;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h ^= w[i];
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 29;
  }
  for (u32 sl = (u32)(h ^ (h >> 32)) & tmask;; sl = (sl + 1) & tmask) {
    const u32 cur = atomicCAS(&table[sl], 0xFFFFFFFFu, g);
    if (cur == 0xFFFFFFFFu) { rep[g] = g; return; }
    u32 o[8];
    ed_key_words(o, pub32, cur);
    bool eq = true;
#pragma unroll
    for (int i = 0; i < 8; ++i) eq &= o[i] == w[i];
    if (eq) { rep[g] = cur; return; }
  }
}
__global__ __launch_bounds__(256) void k_ed_dedupe_assign(u32 n, const uint8_t* pub32, const u32* rep, u32* uid,
                                                          u32* count, u32 capU, uint8_t* kpub32) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  const bool first = g < n && rep[g] == g;
  const uint64_t m = __ballot(first);
  if (m == 0) return;                                  // wave-uniform
  const u32 lane = threadIdx.x & 63u, leader = (u32)__builtin_ctzll(m);
  u32 b0 = 0;
  if (lane == leader) b0 = atomicAdd(count, (u32)__builtin_popcountll(m));
  b0 = (u32)__shfl((int)b0, (int)leader);
  if (!first) return;
  const u32 u = b0 + (u32)__builtin_popcountll(m & ((1ull << lane) - 1ull));
  uid[g] = u;
  if (u < capU) {
    const uint4* p = (const uint4*)(pub32 + (size_t)g * 32);
    uint4* q = (uint4*)(kpub32 + (size_t)u * 32);
    q[0] = p[0];
    q[1] = p[1];
  }
}
__global__ __launch_bounds__(256) void k_ed_dedupe_map(u32 n, const u32* rep, const u32* uid, u32* slot) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n) slot[g] = uid[rep[g]];
}
// item-order verdict bytes -> accept bitmap (words up to ceil(n / 64))
__global__ __launch_bounds__(256) void k_ed_pack_bits(u32 n, const uint8_t* out8, uint64_t* bits) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t m = __ballot(g < n && out8[g] != 0);
  if ((threadIdx.x & 63u) == 0 && g < n) bits[g >> 6] = m;
}

}  // namespace ed
}  // namespace gv

extern "C" hipError_t gvk_ed_group(uint32_t n, const uint8_t* pub32, uint32_t* table, uint32_t tslots, uint32_t* rep,
                                   uint32_t* uid, uint32_t* count, uint32_t capU, uint8_t* kpub32, uint32_t* slot,
                                   hipStream_t st) {
  const dim3 blk(256), grd((n + 255) / 256);
  if (hipMemsetAsync(table, 0xFF, (size_t)tslots * 4, st) != hipSuccess || hipMemsetAsync(count, 0, 4, st) != hipSuccess)
    return hipErrorUnknown;
  hipLaunchKernelGGL(gv::ed::k_ed_dedupe, grd, blk, 0, st, n, pub32, table, tslots - 1, rep);
  hipLaunchKernelGGL(gv::ed::k_ed_dedupe_assign, grd, blk, 0, st, n, pub32, (const uint32_t*)rep, uid, count, capU,
                     kpub32);
  hipLaunchKernelGGL(gv::ed::k_ed_dedupe_map, grd, blk, 0, st, n, (const uint32_t*)rep, (const uint32_t*)uid, slot);
  return hipGetLastError();
}

extern "C" hipError_t gvk_ed_pack_bits(uint32_t n, const uint8_t* out8, uint64_t* bits, hipStream_t st) {
  hipLaunchKernelGGL(gv::ed::k_ed_pack_bits, dim3((n + 255) / 256), dim3(256), 0, st, n, out8, bits);
  return hipGetLastError();
}

extern "C" hipError_t gvk_ed_keyed(const gvk_edk* b, hipStream_t st) {
  if (b->n == 0) return hipSuccess;
  if (b->rb == 6) hipLaunchKernelGGL(gv::ed::k_ed_keyed<6>, dim3((b->n + 255) / 256), dim3(256), 0, st, *b);
  else hipLaunchKernelGGL(gv::ed::k_ed_keyed<4>, dim3((b->n + 255) / 256), dim3(256), 0, st, *b);
  return hipGetLastError();
}

extern "C" hipError_t gvk_ed_keys(const uint8_t* pub32, uint32_t n, uint32_t base, uint32_t* ktab, uint32_t* kpub,
                                  uint32_t* kok, uint32_t* wbase, int rb, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (rb == 6 && !wbase) return hipErrorInvalidValue;     // the radix-64 tables: the split build only
  if (wbase && rb == 6) {                   // chain + table launches (scratch: n * 64 * 36 words)
    hipLaunchKernelGGL(gv::ed::k_ed_keys_chain<6>, dim3((n + 63) / 64), dim3(64), 0, st, pub32, n, base, kpub, kok,
                       wbase);
    hipLaunchKernelGGL(gv::ed::k_ed_keys_tab<6>, dim3((n * gv::ed::EdComb<6>::NW + 255) / 256), dim3(256), 0, st, n,
                       base, ktab, (const uint32_t*)wbase);
  } else if (wbase) {
    hipLaunchKernelGGL(gv::ed::k_ed_keys_chain<4>, dim3((n + 63) / 64), dim3(64), 0, st, pub32, n, base, kpub, kok,
                       wbase);
    hipLaunchKernelGGL(gv::ed::k_ed_keys_tab<4>, dim3((n * 64 + 255) / 256), dim3(256), 0, st, n, base, ktab,
                       (const uint32_t*)wbase);
  } else {
    hipLaunchKernelGGL(gv::ed::k_ed_keys, dim3((n + 63) / 64), dim3(64), 0, st, pub32, n, base, ktab, kpub, kok);
  }
  return hipGetLastError();
}

extern "C" hipError_t gvk_ed_lat(const gvk_edl* b, hipStream_t st) {
  if (b->n == 0) return hipSuccess;
  hipLaunchKernelGGL(gv::ed::k_ed_lat_sl, dim3(b->n), dim3(256), 0, st, *b);
  return hipGetLastError();
}

#if GV_LAT_TRACE
extern "C" int gv_debug_edl_trace(uint64_t* out, int blocks) {
  if (blocks < 0 || blocks > 256) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(gv::ed::g_edl_trace), (size_t)blocks * 8 * 8) == hipSuccess ? 0 : -3;
}
#endif

extern "C" hipError_t gvk_ed_lat_unc(const gvk_edl* b, hipStream_t st) {
  if (b->n == 0) return hipSuccess;
  if (!b->pub32 || !b->btab || !b->out8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gv::ed::k_ed_lat_unc, dim3(b->n), dim3(256), 0, st, *b);
  return hipGetLastError();
}
