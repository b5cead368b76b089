// gv_lat.hip -- the small-batch (CheckTx mempool) latency
// path of the secp256k1 verifier: one fused kernel, the work of each
// signature spread over several lanes and two waves.
//
// Same verdict as the throughput pipeline (gv_kernels.hip) and the reference
// (x/auth/ante/sigverify.go:210 -> tendermint VerifyBytes -> btcec /
// crypto/ecdsa.Verify): identical checks, identical group law; only the
// schedule differs.  A throughput launch gives each signature one lane and
// runs the stages back to back, so a batch of 64 costs the full serial chain
// of one lane (~1 ms).  Here a block of 128 threads takes LAT_SIGS = 16
// signatures:
//   wave 0, lanes 4s..4s+3 (signature s): pubkey decompression (sqrt chain),
//           then the Q and lambda*Q tables in LDS;
//   wave 1, lane s:  range / low-S checks, s^-1 (Fermat, radix-2^29
//           Montgomery), u1 = e w, u2 = r w, GLV split, Booth digits -> LDS.
//   The two chains run concurrently; one barrier.
//   wave 0 ladder: lane 4s + k accumulates ONE of the four partial sums
//           k1q*Q, k2q*(lambda Q), k1g*G, k2g*(lambda G) (125 doublings and
//           <= 26 additions instead of 125 and 66 on one lane), then two
//           cross-lane rounds of complete Jacobian additions combine them and
//           lane 4s runs the final x(R) == r check.
// The field layer is compiled with F29_NCH = 2 (two interleaved mad chains
// per column): a single wave per SIMD waits on every dependent mad, and the
// second chain fills those slots (tools/microbench/fe29_rate.hip, latency
// mode).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "secp_field.cuh"
#include "secp_scalar.cuh"
#include "secp_group29.cuh"
#include "secp_group29x.cuh"
#include "secp_sc29.cuh"
#include "secp_modinv.cuh"
#include "secp_fsl.cuh"
#include "secp_modinv_sl.cuh"
#include "secp_sha256.cuh"

#include "gv_kernels.h"

static_assert(F29_NCH == 2, "gv_lat.hip is built with -DF29_NCH=2");
#if defined(__HIP_DEVICE_COMPILE__) && defined(__AMDGCN_WAVEFRONT_SIZE) && __AMDGCN_WAVEFRONT_SIZE != 64
#error "gv_lat.hip passes table entries between lanes of one wave64"
#endif

namespace gv {

// Q digit width of a shared-state type: kQ6 (the kn arena's 6-bit windows),
// kKW (the wide arena's GV_KW_QW-bit windows), else k4's 5-bit ones.
template <class SH, class = void>
struct lat_q_width {
  static constexpr int qw = SH::kQ6 ? GV_K6_QW : GV_QW;
  static constexpr int qwin = SH::kQ6 ? GV_K6_QWIN : GV_QWIN;
};
template <class SH>
struct lat_q_width<SH, std::void_t<decltype(SH::kKW)>> {
  static constexpr int qw = GV_KW_QW;
  static constexpr int qwin = GV_KW_QWIN;
};

// GV_LAT_TRACE (A/B builds only): per block, wall-clock stamps (100 MHz) of
// the phases -- start, wave 0 prep done, wave 1 scalars done, after the
// barrier, ladder done, combine done, end -- read back with
// gv_debug_lat_trace.  Off in the product build.
#ifndef GV_LAT_TRACE
#define GV_LAT_TRACE 0
#endif
// GV_LAT_SPLITBP: the table's Z back-propagation spread over the signature's
// four lanes (suffix products once, entry scaling in lockstep).
#ifndef GV_LAT_SPLITBP
#define GV_LAT_SPLITBP 1
#endif
// GV_LAT_DIVSTEPS: s^-1 by divsteps (secp_modinv.cuh) instead of the Fermat chain.
#ifndef GV_LAT_DIVSTEPS
#define GV_LAT_DIVSTEPS 1
#endif
#if GV_LAT_TRACE
__device__ uint64_t g_lat_trace[256][8];
#define LAT_STAMP(k) do { if ((threadIdx.x & 63u) == 0 && blockIdx.x < 256) g_lat_trace[blockIdx.x][k] = wall_clock64(); } while (0)
#else
#define LAT_STAMP(k) do { } while (0)
#endif

static __constant__ const u32 kLBeta[8] = {0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u,
                                           0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu};
static __constant__ const u32 kLP[8] = {0xFFFFFC2Fu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                        0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};

struct LatShared {
  static constexpr bool kG5 = false;         // G digits: 20-bit windows (dg)
  static constexpr bool kG24 = false;
  static constexpr bool kQ6 = false;          // Q digits: 5-bit windows (6-bit: the kn arena)
  u32 qtab[GV_LAT_SIGS][2][GV_QTAB_N][18];  // Q, lambda*Q entries: x, y raw 29-bit limbs (effective affine)
  u32 ratio[64][GV_QTAB_N - 1][9];          // per-lane Z-ratio scratch of the table build (raw limbs)
  u32 dq[GV_LAT_SIGS][GV_QWIN];             // packed int16 Q / lambda*Q digits per window
  int dg[GV_LAT_SIGS][GV_GWIN][2];          // G / lambda*G digits
  u32 zq[GV_LAT_SIGS][8];
  u32 r[GV_LAT_SIGS][8];
  u32 okp[GV_LAT_SIGS];                     // pubkey checks passed (wave 0)
  u32 oks[GV_LAT_SIGS];                     // bit 0: scalar checks passed, bit 1: r < p - n (wave 1)
};

// The lanes of one signature hand table entries to each other through LDS
// inside one wave64.  The hardware executes a wave's LDS operations in order;
// the fence + wave barrier make that ordering part of the program (no compiler
// reordering of the LDS stores and loads across this point).
GV_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

GV_DEV u32 be32(const uint8_t* p) {
  return ((u32)p[0] << 24) | ((u32)p[1] << 16) | ((u32)p[2] << 8) | (u32)p[3];
}

GV_DEV void lds_put_ent(u32* e, const fe29& x, const fe29& y) {
#pragma unroll
  for (int i = 0; i < 9; ++i) { e[i] = x.n[i]; e[9 + i] = y.n[i]; }
}
GV_DEV void lds_get_ent(fe29& x, fe29& y, const u32* e) {
#pragma unroll
  for (int i = 0; i < 9; ++i) { x.n[i] = e[i]; y.n[i] = e[9 + i]; }
}

// Wave 0 prep for one signature (all four lanes of it compute; slot 0 stores).
// Table build as build_q_table in gv_kernels.hip (co-Z chain + one
// back-propagation of the Z ratios), into LDS; the back-propagation also
// writes the lambda*Q entry (beta*x, y).
GV_DEV void lat_pubkey_and_tables(LatShared& sh, int sig, int slot, bool live, const uint8_t* pub33) {
  const uint8_t* p = pub33;
  u32 pre = live ? p[0] : 0u;
  fe x8;
#pragma unroll
  for (int i = 0; i < 8; ++i) x8.v[i] = live ? be32(p + 1 + 4 * (7 - i)) : 0u;
  bool ok = live && (pre & 0xFEu) == 0x02u;
  {
    u32 br = 0, d;
#pragma unroll
    for (int i = 0; i < 8; ++i) d = __builtin_subc(x8.v[i], kLP[i], br, &br);
    (void)d;
    ok &= (br != 0);                                    // x < p
  }
  fe y8;
  {
    fe29 x29, c, y29, y2, seven;
    f29_from_words(x29, x8.v);
    f29_sqr(c, x29);
    f29_mul(c, c, x29);
    f29_set_u32(seven, 7);
    f29_add(c, c, seven);                               // x^3 + 7
    f29_sqrt_candidate(y29, c);
    f29_sqr(y2, y29);
    ok &= f29_equal(y2, c);                             // "invalid square root"
    f29_to_words(y8.v, y29);
  }
  if ((y8.v[0] & 1u) != (pre & 1u)) fe_neg(y8, y8);
  fe_normalize(y8);
  LAT_STAMP(7);
  if (!ok) {                                          // harmless stand-in point: G
    const u32 gx[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                       0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
    const u32 gy[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                       0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
#pragma unroll
    for (int i = 0; i < 8; ++i) { x8.v[i] = gx[i]; y8.v[i] = gy[i]; }
  }
  const bool st = slot == 0;
  u32 (*qt)[18] = sh.qtab[sig][0];
  u32 (*lt)[18] = sh.qtab[sig][1];
  u32 (*qr)[9] = sh.ratio[sig * 4 + slot];
  fe29 qx, qy, X1, Y1, X2, Y2, t, u;
  f29_from_words(qx, x8.v);
  f29_from_words(qy, y8.v);
  {
    fe29 B, E, L, M;
    f29_sqr(B, qx);
    f29_sqr(E, qy);
    f29_sqr(L, E);
    f29_add(t, qx, E);
    f29_sqr(t, t);
    f29_sub<1>(t, t, B);
    f29_sub_norm<1>(t, t, L);
    f29_shl_norm<1>(X1, t);                           // S = 4xy^2
    f29_mul3_norm(M, B);
    f29_sqr(t, M);
    f29_add(u, X1, X1);
    f29_sub_norm<2>(X2, t, u);                        // 2Q.x
    f29_shl_norm<3>(Y1, L);                           // 8y^4
    f29_sub<1>(t, X1, X2);
    f29_mul(t, M, t);
    f29_sub_norm<1>(Y2, t, Y1);                       // 2Q.y
  }
  if (st) { lds_put_ent(qt[0], X1, Y1); lds_put_ent(qt[1], X2, Y2); }
  for (int m = 2; m < GV_QTAB_N; ++m) {
    fe29 h, rr, c, w1, w2, d, a1;
    f29_sub_norm<1>(h, X1, X2);
#pragma unroll
    for (int i = 0; i < 9; ++i) qr[m - 2][i] = h.n[i];  // lane-private
    f29_sub_norm<1>(rr, Y1, Y2);
    f29_sqr(c, h);
    f29_mul(w1, X1, c);
    f29_mul(w2, X2, c);
    f29_sqr(d, rr);
    f29_sub<1>(t, w1, w2);
    f29_mul(a1, Y1, t);
    f29_add(u, w1, w2);
    f29_sub_norm<2>(X2, d, u);
    f29_sub<1>(t, w1, X2);
    f29_mul(t, rr, t);
    f29_sub_norm<1>(Y2, t, a1);
    X1 = w1;
    Y1 = a1;
    if (st) lds_put_ent(qt[m], X2, Y2);
  }
  wave_lds_sync();                                    // slot 0's entries -> the other lanes
  // Back-propagation: entry m-1 scaled to the last entry's Z (as in
  // build_q_table: entry index j lives on Z_max(j,1), ratio[k] = Z_(k+2) /
  // Z_(k+1)).  Every lane reads the entries its signature's slot-0 lane stored
  // above (same wave, earlier instructions: LDS executes one wave's operations
  // in order); the lambda*Q entry (beta*x, y) is written alongside.
  fe29 acc, beta;
  {
    u32 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = kLBeta[i];
    f29_from_words(beta, w);
  }
#if GV_LAT_SPLITBP
  // (1) the suffix products acc_m = prod_{k=m..15} ratio_k, m = 15..2, on every
  // lane alike; slot 0 overwrites its ratio scratch with them (read back by the
  // other lanes of the signature: same wave, program order).
  {
    u32 (*qr0)[9] = sh.ratio[sig * 4];
#pragma unroll 1
    for (int m = GV_QTAB_N - 1; m >= 2; --m) {
      fe29 ratio;
#pragma unroll
      for (int i = 0; i < 9; ++i) ratio.n[i] = qr[m - 2][i];     // Z_m / Z_(m-1)
      if (m == GV_QTAB_N - 1) acc = ratio;
      else f29_mul(acc, acc, ratio);
      if (st) {
#pragma unroll
        for (int i = 0; i < 9; ++i) qr0[m - 2][i] = acc.n[i];
      }
    }
    wave_lds_sync();                                  // slot 0's suffix products -> the other lanes
    // (2) lane 4s + k scales entries k, k+4, k+8, k+12 in lockstep: entry e
    // (on Z_max(e,1)) times acc_(e+1)^2, acc_(e+1)^3 (entry 0 uses acc_2, the
    // last entry is already on Z_15), and writes its lambda*Q entry.
#pragma unroll 1
    for (int j = 0; j < GV_QTAB_N / 4; ++j) {
      const int e = 4 * j + slot;
      fe29 x, y, a, a2, a3;
      lds_get_ent(x, y, qt[e]);
      if (e == GV_QTAB_N - 1) f29_set_u32(a, 1);
      else if (e == 0) a = acc;
      else {
#pragma unroll
        for (int i = 0; i < 9; ++i) a.n[i] = qr0[e - 1][i];    // acc_(e+1)
      }
      f29_sqr(a2, a);
      {
        fe29 o[2];
        const fe29 xa[2] = {a2, x}, ya[2] = {a, a2};
        f29_multi<false, false>(o, xa, ya);
        a3 = o[0]; x = o[1];
      }
      f29_mul(y, y, a3);
      f29_mul(t, x, beta);
      lds_put_ent(qt[e], x, y);
      lds_put_ent(lt[e], t, y);
    }
  }
#else
  for (int m = GV_QTAB_N; m >= 1; --m) {
    fe29 x, y;
    lds_get_ent(x, y, qt[m - 1]);
    if (m < GV_QTAB_N) {
      if (m >= 2) {
        fe29 ratio;
#pragma unroll
        for (int i = 0; i < 9; ++i) ratio.n[i] = qr[m - 2][i];   // Z_m / Z_(m-1)
        if (m == GV_QTAB_N - 1) acc = ratio;
        else f29_mul(acc, acc, ratio);
      }
      fe29 a2, a3;
      f29_sqr(a2, acc);
      f29_mul(a3, a2, acc);
      f29_mul(x, x, a2);
      f29_mul(y, y, a3);
      if (st) lds_put_ent(qt[m - 1], x, y);
    }
    f29_mul(t, x, beta);
    if (st) lds_put_ent(lt[m - 1], t, y);
  }
#endif
  f29_add(t, qy, qy);
  f29_mul(t, t, acc);                                 // Z_15 = 2y * prod(ratios)
  if (st) {
    u32 w[8];
    f29_to_words(w, t);
#pragma unroll
    for (int i = 0; i < 8; ++i) sh.zq[sig][i] = w[i];
    sh.okp[sig] = ok ? 1u : 0u;
  }
}


// Wave 0 prep for a keyed signature (gv_keys_load): the Q table comes from the
// key arena row (built once per key by k_keys_chain + k_keys_tables, same effective-affine
// form and Z), so no square root and no table build.  Lane 4s + k copies
// entries k, k+4, k+8, k+12 and forms their lambda*Q entries (beta*x, y).
GV_DEV void lat_keyed_tables(LatShared& sh, int sig, int slot, bool live, u32 kslot, const u32* kqt,
                             const u32* kzq, const u32* kok, u32 kC, u32 kcount) {
  u32 sl = live ? kslot : 0xFFFFFFFFu;
  bool ok = sl < kcount;
  if (!ok) sl = 0;                                    // the arena always holds slot 0's memory
  ok = ok && kok[sl] != 0u;
  fe29 beta;
  {
    u32 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = kLBeta[i];
    f29_from_words(beta, w);
  }
#pragma unroll 1
  for (int m = slot; m < GV_QTAB_N; m += 4) {
    const uint4* p = (const uint4*)(kqt + ((size_t)sl * GV_QTAB_N + m) * GV_QENT_WORDS);
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3], e = p[4];
    fe29 x, y, t;
    x.n[0] = a.x; x.n[1] = a.y; x.n[2] = a.z; x.n[3] = a.w;
    x.n[4] = b.x; x.n[5] = b.y; x.n[6] = b.z; x.n[7] = b.w;
    x.n[8] = c.x; y.n[0] = c.y; y.n[1] = c.z; y.n[2] = c.w;
    y.n[3] = d.x; y.n[4] = d.y; y.n[5] = d.z; y.n[6] = d.w;
    y.n[7] = e.x; y.n[8] = e.y;
    lds_put_ent(sh.qtab[sig][0][m], x, y);
    f29_mul(t, x, beta);
    lds_put_ent(sh.qtab[sig][1][m], t, y);
  }
  if (slot == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) sh.zq[sig][i] = kzq[(size_t)i * kC + sl];
    sh.okp[sig] = ok ? 1u : 0u;
  }
}

// The keyed 16-lane schedule's shared state (k_verify_lat16).
struct Lat16Shared {
  static constexpr bool kG5 = true;          // G digits: 5-bit windows like Q (dg5)
  static constexpr bool kG24 = false;
  static constexpr bool kQ6 = false;          // Q digits: 5-bit windows (6-bit: the kn arena)
  u32 dq[GV_LAT16_SIGS][GV_QWIN];            // packed int16 Q / lambda*Q digits per window
  u32 dg5[GV_LAT16_SIGS][GV_QWIN];           // packed int16 G / lambda*G digits per window
  u32 r[GV_LAT16_SIGS][8];
  u32 oks[GV_LAT16_SIGS];
  u32 res[GV_LAT16_SIGS];
};

// The scalar chain of one signature (one lane): range / low-S checks, s^-1,
// u1, u2, GLV split, Booth digits -> sh.  VAR: called by a whole wave with
// the same signature in every lane (the sliced kernels); s^-1 by the
// variable-time divsteps with the state vectors sliced over the lanes
// (s30_modinv_sl).  Otherwise one signature per lane, lockstep divsteps.
template <bool VAR = false, class SH, class GetE>
GV_DEV void lat_scalars_e(SH& sh, int sig, bool live, const uint8_t* sig64, GetE get_e) {
  u32 r[8], s[8], e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r[i] = live ? be32(sig64 + 4 * (7 - i)) : 0u;
    s[i] = live ? be32(sig64 + 32 + 4 * (7 - i)) : 0u;
  }
  bool ok = live;
  ok &= !u256_is_zero(r);
  ok &= !u256_geq(r, kN);
  ok &= !u256_is_zero(s);
  ok &= u256_geq(kHalfN, s);                // tendermint low-S: s <= N/2
  const bool r_small = !u256_geq(r, kPminusN);
  if (!ok) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { s[i] = (i == 0) ? 1u : 0u; r[i] = 0u; }
  }
  u32 u1[8], u2[8];
  {
    sc29 s29, w, e29, r29, t;
#if GV_LAT_DIVSTEPS
    u32 si[8];                              // s^-1 by divsteps: ~4x shorter chain than Fermat
    if constexpr (VAR) s30_modinv_sl(si, s, fsl_consts());   // whole wave, limbs over lanes
    else s30_modinv(si, s, [](bool done) { return __all(done) != 0; });
    sc29_from_words(s29, si);
    sc29_to_mont(w, s29);                   // s^-1 (Montgomery form)
#else
    sc29 sm;
    sc29_from_words(s29, s);
    sc29_to_mont(sm, s29);
    sc29_inv(w, sm);                        // s^-1 (Montgomery form), Fermat chain
#endif
    // e is needed only from here: a message digest computed by another wave
    // meanwhile (get_e may wait for it)
    get_e(e);
    if (!live) {
#pragma unroll
      for (int i = 0; i < 8; ++i) e[i] = 0u;
    }
    sc_reduce_once(e);                      // e mod n
    if (!ok) {
#pragma unroll
      for (int i = 0; i < 8; ++i) e[i] = 0u;
    }
    sc29_from_words(e29, e);
    sc29_from_words(r29, r);
    sc29_mul(t, e29, w);
    sc29_to_words(u1, t);                   // e * s^-1
    sc29_mul(t, r29, w);
    sc29_to_words(u2, t);                   // r * s^-1
  }
  u32 k1g[4], k2g[4], k1q[4], k2q[4], n1g, n2g, n1q, n2q;
  glv_split(k1g, n1g, k2g, n2g, u1);
  glv_split(k1q, n1q, k2q, n2q, u2);
  if (!ok) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { k1g[i] = k2g[i] = k1q[i] = k2q[i] = 0u; }
  }
  constexpr int QW = lat_q_width<SH>::qw, QWIN = lat_q_width<SH>::qwin;
#pragma unroll
  for (int win = 0; win < QWIN; ++win) {
    int d0 = booth_digit<QW>(k1q, win), d1 = booth_digit<QW>(k2q, win);
    if (n1q) d0 = -d0;
    if (n2q) d1 = -d1;
    sh.dq[sig][win] = ((u32)d0 & 0xFFFFu) | ((u32)d1 << 16);
  }
  if constexpr (SH::kG24) {
    // G on the unsplit u1: 11 signed 24-bit windows (the k6 tables' digits)
    if (!ok) {
#pragma unroll
      for (int i = 0; i < 8; ++i) u1[i] = 0u;
    }
#pragma unroll
    for (int j = 0; j < GV_K6_GWIN; ++j) sh.dg24[sig][j] = booth_digit8<GV_K6_GW>(u1, j);
  } else if constexpr (SH::kG5) {
#pragma unroll
    for (int win = 0; win < GV_QWIN; ++win) {
      int d2 = booth_digit<GV_QW>(k1g, win), d3 = booth_digit<GV_QW>(k2g, win);
      if (n1g) d2 = -d2;
      if (n2g) d3 = -d3;
      sh.dg5[sig][win] = ((u32)d2 & 0xFFFFu) | ((u32)d3 << 16);
    }
  } else {
#pragma unroll
    for (int j = 0; j < GV_GWIN; ++j) {
      int d2 = booth_digit<GV_GW>(k1g, j), d3 = booth_digit<GV_GW>(k2g, j);
      if (n1g) d2 = -d2;
      if (n2g) d3 = -d3;
      sh.dg[sig][j][0] = d2;
      sh.dg[sig][j][1] = d3;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) sh.r[sig][i] = r[i];
  sh.oks[sig] = (ok ? 1u : 0u) | (r_small ? 2u : 0u);
}

// e from the digest bytes (dig32), the SHA state words (eh) or the SoA rows
// written by k_sha256 (e_soa, stride C)
template <bool VAR = false, class SH>
GV_DEV void lat_scalars(SH& sh, int sig, bool live, const uint8_t* sig64, const uint8_t* dig32,
                        const u32* e_soa, u32 C, u32 gi, const u32* eh = nullptr) {
  lat_scalars_e<VAR>(sh, sig, live, sig64, [&](u32 e[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      e[i] = !live ? 0u : eh ? eh[7 - i] : dig32 ? be32(dig32 + 4 * (7 - i)) : e_soa[(size_t)i * C + gi];
  });
}

GV_DEV void shfl_xor_gej(gej29& o, bool& oinf, const gej29& a, bool ainf, int m) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    o.x.n[i] = (u32)__shfl_xor((int)a.x.n[i], m, 64);
    o.y.n[i] = (u32)__shfl_xor((int)a.y.n[i], m, 64);
    o.z.n[i] = (u32)__shfl_xor((int)a.z.n[i], m, 64);
  }
  oinf = __shfl_xor((int)ainf, m, 64) != 0;
}

// GV_LAT_FUSED: the latency ladders on the fused formulas (secp_group29x.cuh,
// two mad chains per column in this translation unit: F29X_NCH = 2); 0 = the
// secp_group29.cuh formulas with lockstep product pairs.
#ifndef GV_LAT_FUSED
#define GV_LAT_FUSED 1
#endif
GV_DEV void lat_double(gej29& acc) {
#if GV_LAT_FUSED
  gej29x_double(acc, acc);
#else
  gej29_double(acc, acc);
#endif
}
// acc += (x, y), an affine point of the lane's curve (y magnitude <= 2); an
// infinite accumulator takes the point.
GV_DEV void lat_add_affine(gej29& acc, bool& inf, const fe29& x, const fe29& y) {
#if GV_LAT_FUSED
  if (inf) {
    acc.x = x;
    f29_norm(acc.y, y);
    f29_set_u32(acc.z, 1);
    inf = false;
  } else {
    gej29x_add_scaled(acc, inf, x, y, acc.z);
  }
#else
  fe29 az, z2, u2, s2;
  if (inf) f29_set_u32(az, 1);
  else az = acc.z;
  f29_sqr(z2, az);
  {
    fe29 o[2];
    const fe29 xa[2] = {x, z2}, ya[2] = {z2, az};
    f29_multi<false, false>(o, xa, ya);
    u2 = o[0]; z2 = o[1];
  }
  f29_mul(s2, y, z2);
  if (inf) {
    acc.x = u2; acc.y = s2; f29_set_u32(acc.z, 1); inf = false;
  } else {
    gej29_add_tail(acc, inf, u2, s2);
  }
#endif
}


// One block = GV_LAT_SIGS signatures, 128 threads.  Inputs: AoS bytes as in
// gv_verify_digests; e from dig32 (digest path) or from the SoA rows e_soa
// written by k_sha256 (message path, stride C).  Output: 16 verdict bits per
// block, bits16[block] (the u64 bitmap viewed as u16 words).
__global__ __launch_bounds__(128) void k_verify_lat(const u32* gtab, const uint8_t* pub33,
                                                     const uint8_t* sig64, const uint8_t* dig32,
                                                     const u32* e_soa, u32 C, u32 n, uint16_t* bits16,
                                                     const u32* kslot, const u32* kqt, const u32* kzq,
                                                     const u32* kok, u32 kC, u32 kcount) {
  __shared__ LatShared sh;
  const u32 wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  if (wave == 0) LAT_STAMP(0);
  if (wave == 0) {
    const int sig = lane >> 2, slot = lane & 3;
    const u32 gi = blockIdx.x * GV_LAT_SIGS + sig;
    const bool live = gi < n;
    if (kslot)                                        // keyed batch: tables from the key arena
      lat_keyed_tables(sh, sig, slot, live, live ? kslot[gi] : 0u, kqt, kzq, kok, kC, kcount);
    else
      lat_pubkey_and_tables(sh, sig, slot, live, pub33 + (size_t)(live ? gi : 0) * 33u);
  } else if (lane < GV_LAT_SIGS) {
    const u32 gi = blockIdx.x * GV_LAT_SIGS + lane;
    const bool live = gi < n;
    const u32 gs = live ? gi : 0u;
    lat_scalars(sh, lane, live, sig64 + (size_t)gs * 64u, dig32 ? dig32 + (size_t)gs * 32u : nullptr,
                e_soa, C, gs);
  }
  if (wave == 0) LAT_STAMP(1); else LAT_STAMP(2);
  __syncthreads();
  if (wave != 0) return;
  LAT_STAMP(3);

  // ---- ladder: lane 4s + slot accumulates one of the four partial sums
  const int sig = lane >> 2, slot = lane & 3;
  gej29 acc;
  f29_set_zero(acc.x); f29_set_zero(acc.y); f29_set_zero(acc.z);
  bool inf = true;
#pragma unroll 1
  for (int win = GV_QWIN - 1; win >= 0; --win) {
    if (win != GV_QWIN - 1) {
#pragma unroll 1
      for (int d = 0; d < GV_QW; ++d) lat_double(acc);
    }
    const bool gwin = (win % GV_GSTEP) == 0;          // block-uniform
    const u32 dq = sh.dq[sig][win];
    int d;
    if (slot < 2) d = slot == 0 ? ((int)(dq << 16) >> 16) : ((int)dq >> 16);
    else d = gwin ? sh.dg[sig][win / GV_GSTEP][slot - 2] : 0;
    if (d != 0) {
      const u32 e = (u32)((d < 0 ? -d : d) - 1);
      fe29 x, y;
      if (slot < 2) {
        lds_get_ent(x, y, sh.qtab[sig][slot][e]);
      } else {
        const uint4* p = (const uint4*)(gtab + ((size_t)(slot == 3 ? GV_GTAB_N : 0) + e) * 16);
        uint4 a = p[0], b = p[1], c = p[2], dd = p[3];
        u32 wx[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        u32 wy[8] = {c.x, c.y, c.z, c.w, dd.x, dd.y, dd.z, dd.w};
        f29_from_words(x, wx);
        f29_from_words(y, wy);
      }
      if (d < 0) f29_neg<1>(y, y);
      // Q slots live on the isomorphic curve of the shared table Z, G slots on
      // the real curve: either way the entry is affine on the lane's curve.
      lat_add_affine(acc, inf, x, y);
    }
  }

  LAT_STAMP(4);
  // ---- combine: Q-slot points back to the real curve (Z *= zq), then two
  // rounds of complete additions across the signature's four lanes.
  {
    u32 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = sh.zq[sig][i];
    fe29 zq;
    f29_from_words(zq, w);
    if (slot >= 2) f29_set_u32(zq, 1);
    f29_mul(acc.z, acc.z, zq);
  }
  gej29 other;
  bool oinf;
  shfl_xor_gej(other, oinf, acc, inf, 1);
  gej29_add_gej(acc, inf, acc, inf, other, oinf);
  shfl_xor_gej(other, oinf, acc, inf, 2);
  gej29_add_gej(acc, inf, acc, inf, other, oinf);

  LAT_STAMP(5);
  // ---- final check (as k_ecmult): x(R) mod n == r, without inversion
  const u32 fl = sh.oks[sig];
  bool ok = (fl & 1u) && sh.okp[sig] && !inf;
  fe29 zz, rf, t;
  f29_sqr(zz, acc.z);
  u32 rw[8], X[8], tw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) rw[i] = sh.r[sig][i];
  f29_from_words(rf, rw);
  f29_mul(t, rf, zz);
  f29_to_words(X, acc.x);
  f29_to_words(tw, t);
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) eq &= (X[i] == tw[i]);
  if (!eq && (fl & 2u)) {
    u32 rn[8], c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) rn[i] = __builtin_addc(rw[i], kN[i], c, &c);
    f29_from_words(rf, rn);
    f29_mul(t, rf, zz);
    f29_to_words(tw, t);
    eq = true;
#pragma unroll
    for (int i = 0; i < 8; ++i) eq &= (X[i] == tw[i]);
  }
  ok &= eq;
  const uint64_t m = __ballot(ok && slot == 0);
  if (lane == 0) {
    u32 b16 = 0;
#pragma unroll
    for (int s2 = 0; s2 < GV_LAT_SIGS; ++s2) b16 |= (u32)((m >> (4 * s2)) & 1u) << s2;
    bits16[blockIdx.x] = (uint16_t)b16;
    LAT_STAMP(6);
    if (blockIdx.x == gridDim.x - 1) {           // zero the rest of the last 64-bit word
      for (u32 k = blockIdx.x + 1; (k & 3u) != 0u; ++k) bits16[k] = 0;
    }
  }
}

// ---------------------------------------------------------------------------
// Keyed small batches (C5 with the account's key resident, gv_keys_load):
// 16 lanes per signature, GV_LAT16_SIGS = 8 signatures per 128-thread block.
// Lane (s, j): part = j & 3 picks k1q*Q, k2q*(lambda Q), k1g*G or k2g*(lambda
// G); group = j >> 2 picks the windows [0,7), [7,14), [14,20) or [20,26) of
// that 128-bit half, against the table of 2^(5 w0) times the base (the key
// arena's group tables for Q, glat for G).  So each lane runs at most 30
// doublings and 7 table additions instead of 125 and 26; four cross-lane
// rounds of complete Jacobian additions combine the 16 partial sums and lane
// j == 0 runs the same inversion-free final check.  The scalar chain runs
// first, on lane j == 0 of each signature (the tables need no preparation).
static __constant__ const int kL16Win[GV_LGRP + 1] = {0, 7, 14, 20, GV_QWIN};

__global__ __launch_bounds__(128) void k_verify_lat16(const gvk_lat b) {
  __shared__ Lat16Shared sh;
  const u32 tid = threadIdx.x, sig = tid >> 4, j = tid & 15u;
  const u32 gi = blockIdx.x * GV_LAT16_SIGS + sig;
  const bool live = gi < b.n;
  const u32 gs = live ? gi : 0u;
  u32 sl = live ? b.kslot[gs] : 0xFFFFFFFFu;
  bool kok = sl < b.kcount;
  if (!kok) sl = 0;                                     // the arena always holds slot 0's memory
  kok = kok && b.kok[sl] != 0u;
  if (j == 0)
    lat_scalars(sh, (int)sig, live, b.sig64 + (size_t)gs * 64u, b.dig32 ? b.dig32 + (size_t)gs * 32u : nullptr,
                b.msg_blob ? (const u32*)b.e_soa : nullptr, b.C, gs);
  __syncthreads();

  const int part = (int)(j & 3u), grp = (int)(j >> 2);
  const int w_lo = kL16Win[grp], w_hi = kL16Win[grp + 1] - 1;
  fe29 beta;
  {
    u32 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = kLBeta[i];
    f29_from_words(beta, w);
  }
  const u32* qrow = grp == 0 ? b.kqt + (size_t)sl * GV_QTAB_N * GV_QENT_WORDS
                             : b.kqt2 + ((size_t)sl * GV_KEY2_TABLES + (grp - 1)) * GV_QTAB_N * GV_QENT_WORDS;
  const u32* grow = b.glat + (size_t)(grp * 2 + (part & 1)) * GV_QTAB_N * 16;
  gej29 acc;
  f29_set_zero(acc.x); f29_set_zero(acc.y); f29_set_zero(acc.z);
  bool inf = true;
#pragma unroll 1
  for (int win = w_hi; win >= w_lo; --win) {
    if (win != w_hi) {
#pragma unroll 1
      for (int d = 0; d < GV_QW; ++d) lat_double(acc);
    }
    const u32 dw = part < 2 ? sh.dq[sig][win] : sh.dg5[sig][win];
    const int d = (part & 1) == 0 ? ((int)(dw << 16) >> 16) : ((int)dw >> 16);
    if (d != 0) {
      const u32 e = (u32)((d < 0 ? -d : d) - 1);
      fe29 x, y;
      if (part < 2) {                                   // Q / lambda Q: arena row, 29-bit limbs
        const uint4* p = (const uint4*)(qrow + (size_t)e * GV_QENT_WORDS);
        const uint4 a = p[0], bb = p[1], c = p[2], dd = p[3], ee = p[4];
        x.n[0] = a.x; x.n[1] = a.y; x.n[2] = a.z; x.n[3] = a.w;
        x.n[4] = bb.x; x.n[5] = bb.y; x.n[6] = bb.z; x.n[7] = bb.w;
        x.n[8] = c.x; y.n[0] = c.y; y.n[1] = c.z; y.n[2] = c.w;
        y.n[3] = dd.x; y.n[4] = dd.y; y.n[5] = dd.z; y.n[6] = dd.w;
        y.n[7] = ee.x; y.n[8] = ee.y;
        if (part == 1) f29_mul(x, x, beta);             // lambda Q = (beta x, y), same Z
      } else {                                          // G / lambda G: affine words
        const uint4* p = (const uint4*)(grow + (size_t)e * 16);
        const uint4 a = p[0], bb = p[1], c = p[2], dd = p[3];
        u32 wx[8] = {a.x, a.y, a.z, a.w, bb.x, bb.y, bb.z, bb.w};
        u32 wy[8] = {c.x, c.y, c.z, c.w, dd.x, dd.y, dd.z, dd.w};
        f29_from_words(x, wx);
        f29_from_words(y, wy);
      }
      if (d < 0) f29_neg<1>(y, y);
      lat_add_affine(acc, inf, x, y);
    }
  }
  // Q parts live on the isomorphic curve of their table's Z: back to the real curve
  if (part < 2) {
    const u32* zrow = grp == 0 ? b.kzq : b.kzq2 + (size_t)(grp - 1) * 8 * b.kC;
    u32 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = zrow[(size_t)i * b.kC + sl];
    fe29 zq;
    f29_from_words(zq, w);
    f29_mul(acc.z, acc.z, zq);
  }
  gej29 other;
  bool oinf;
#pragma unroll 1
  for (int m = 1; m < 16; m <<= 1) {                    // 16 partial sums -> lane j == 0
    shfl_xor_gej(other, oinf, acc, inf, m);
    gej29_add_gej(acc, inf, acc, inf, other, oinf);
  }
  if (j == 0) {
    const u32 fl = sh.oks[sig];
    bool ok = (fl & 1u) && kok && !inf;
    fe29 zz, rf, t;
    f29_sqr(zz, acc.z);
    u32 rw[8], X[8], tw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) rw[i] = sh.r[sig][i];
    f29_from_words(rf, rw);
    f29_mul(t, rf, zz);
    f29_to_words(X, acc.x);
    f29_to_words(tw, t);
    bool eq = true;
#pragma unroll
    for (int i = 0; i < 8; ++i) eq &= (X[i] == tw[i]);
    if (!eq && (fl & 2u)) {
      u32 rn[8], c = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) rn[i] = __builtin_addc(rw[i], kN[i], c, &c);
      f29_from_words(rf, rn);
      f29_mul(t, rf, zz);
      f29_to_words(tw, t);
      eq = true;
#pragma unroll
      for (int i = 0; i < 8; ++i) eq &= (X[i] == tw[i]);
    }
    sh.res[sig] = (ok && eq) ? 1u : 0u;
  }
  __syncthreads();
  if (tid == 0) {
    u32 b8 = 0;
#pragma unroll
    for (int q = 0; q < GV_LAT16_SIGS; ++q) b8 |= sh.res[q] << q;
    uint8_t* bits8 = (uint8_t*)b.bits;
    bits8[blockIdx.x] = (uint8_t)b8;
    if (blockIdx.x == gridDim.x - 1)                    // zero the rest of the last 64-bit word
      for (u32 k = blockIdx.x + 1; (k & 7u) != 0u; ++k) bits8[k] = 0;
  }
}

// ---------------------------------------------------------------------------
// Pub33 small batches on the limb-sliced field layer (secp_fsl.cuh): ONE
// signature per 128-thread block.  Wave 0 does all the field work with one
// element per 16-lane DPP row -- the four rows decompress the key (sqrt chain)
// and build the Q table together, then row r accumulates the partial sum
// r of {k1q Q, k2q lambda Q, k1g G, k2g lambda G} over the same 125-doubling
// Booth ladder as k_verify_lat, and two cross-row rounds of complete
// additions combine them.  Wave 1 lane 0 runs the scalar chain (lat_scalars)
// concurrently, on its own SIMD.  A sliced product costs ~0.14 us on a lone
// wave against ~0.37 us for the one-lane layer (profiles/r02/fsl), so the
// sqrt chain, the table and the ladder all shorten ~2.5x.  Same checks, same
// group law, same verdict as k_verify_lat.  Verdict bits: atomicOr into the
// bitmap (zeroed by the launcher).
struct LatSlShared {
  static constexpr bool kG5 = false;         // G digits: 20-bit windows (dg)
  static constexpr bool kG24 = false;
  static constexpr bool kQ6 = false;          // Q digits: 5-bit windows (6-bit: the kn arena)
  u32 qtab[2][GV_QTAB_N][18];               // Q, lambda*Q entries: x, y sliced limbs (effective affine)
  u32 ratio[GV_QTAB_N - 1][9];              // Z ratios, then their suffix products
  u32 dq[1][GV_QWIN];
  int dg[1][GV_GWIN][2];
  u32 r[1][8];
  u32 oks[1];
  u32 zq[16];                               // Z of the tables' curve, sliced
  u32 okp;                                  // ParsePubKey verdict
  u32 pt[3][16];                            // wave 2's sum (x, y, z sliced)
  u32 pinf;
};

// Key decompression (btcec ParsePubKey): the ParsePubKey verdict and (x, y),
// with G standing in for an invalid key.
GV_DEV bool lat_sl_decompress(fe& x8, fe& y8, const gvk_lat& b, u32 gi, const fslk& k) {
  const u32 L = k.L;
  // ---- pubkey: btcec ParsePubKey / decompressPoint
  const uint8_t* p = b.pub33 + (size_t)gi * 33u;
  const u32 pre = p[0];
#pragma unroll
  for (int i = 0; i < 8; ++i) x8.v[i] = be32(p + 1 + 4 * (7 - i));
  bool ok = (pre & 0xFEu) == 0x02u;
  {
    u32 br = 0, d;
#pragma unroll
    for (int i = 0; i < 8; ++i) d = __builtin_subc(x8.v[i], kLP[i], br, &br);
    (void)d;
    ok &= (br != 0);                                    // x < p
  }
  {
    const u32 xs = fsl_from_words(x8.v, k);
    const u32 c = fsl_mul(fsl_sqr(xs, k), xs, k) + (L == 0u ? 7u : 0u);   // x^3 + 7
    const u32 y = fsl_sqrt_candidate(c, k);
    u32 w1[8], w2[8];
    fsl_to_words(w1, fsl_sqr(y, k));
    fsl_to_words(w2, c);
    u32 df = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) df |= w1[i] ^ w2[i];
    ok &= df == 0u;                                     // "invalid square root"
    fsl_to_words(y8.v, y);
  }
  if ((y8.v[0] & 1u) != (pre & 1u)) fe_neg(y8, y8);
  fe_normalize(y8);
  LAT_STAMP(1);                                         // trace builds: key decompressed
  if (!ok) {                                            // harmless stand-in point: G
    const u32 gx[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                       0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
    const u32 gy[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                       0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
#pragma unroll
    for (int i = 0; i < 8; ++i) { x8.v[i] = gx[i]; y8.v[i] = gy[i]; }
  }
  return ok;
}

// Q / lambda*Q tables of the point (qx, qy) into LDS and zq (Z of the
// tables' curve), for a whole wave.
template <class SH>
GV_DEV void lat_sl_tables(SH& sh, u32 qx, u32 qy, const fslk& k) {
  const u32 row = (threadIdx.x >> 4) & 3u, L = k.L;
  const bool lo = L < 9u;
  // ---- Q table: co-Z chain (as build_q_table / lat_pubkey_and_tables), row 0 stores
  const bool st = row == 0u && lo;
  u32 X1, Y1, X2, Y2;
  {
    const u32 E = fsl_sqr(qy, k);                       // y^2
    X1 = fsl_mul(qx << 2, E, k);                        // S = 4 x y^2
    const u32 M = fsl_norm(fsl_sqr(qx, k) * 3u, k);     // 3 x^2
    X2 = fsl_mul_plus(M, M, k.big8 - ((u64)X1 << 1), k);               // 2Q.x = M^2 - 2S
    Y1 = fsl_norm(fsl_mul(E << 1, E << 1, k) << 1, k);  // 8 y^4
    Y2 = fsl_mul_plus(M, X1 + k.bias - X2, (u64)(k.bias - Y1), k);     // 2Q.y = M (S - X2) - 8y^4
  }
  if (st) {
    sh.qtab[0][0][L] = X1; sh.qtab[0][0][9 + L] = Y1;
    sh.qtab[0][1][L] = X2; sh.qtab[0][1][9 + L] = Y2;
  }
#pragma unroll 1
  for (int m = 2; m < GV_QTAB_N; ++m) {
    const u32 h = fsl_sub(X1, X2, k);
    if (st) sh.ratio[m - 2][L] = h;                     // Z_m / Z_(m-1)
    const u32 rr = fsl_sub(Y1, Y2, k);
    const u32 cc = fsl_sqr(h, k);
    const u32 w1 = fsl_mul(X1, cc, k), w2 = fsl_mul(X2, cc, k);
    const u32 a1 = fsl_mul(Y1, w1 + k.bias - w2, k);
    X2 = fsl_mul_plus(rr, rr, k.big8 - (u64)w1 - (u64)w2, k);
    Y2 = fsl_mul_plus(rr, w1 + k.bias - X2, (u64)(k.bias - a1), k);
    X1 = w1;
    Y1 = a1;
    if (st) { sh.qtab[0][m][L] = X2; sh.qtab[0][m][9 + L] = Y2; }
  }
  wave_lds_sync();
  // back-propagation: suffix products acc_m = prod_{j=m..15} ratio_j (every
  // row alike, row 0 overwrites the ratios with them), then row r scales
  // entries r, r+4, r+8, r+12 to the last entry's Z and writes their
  // lambda*Q entries (beta x, y)
  u32 acc = 0;
#pragma unroll 1
  for (int m = GV_QTAB_N - 1; m >= 2; --m) {
    const u32 ratio = lo ? sh.ratio[m - 2][L] : 0u;
    acc = m == GV_QTAB_N - 1 ? ratio : fsl_mul(acc, ratio, k);
    if (st) sh.ratio[m - 2][L] = acc;
  }
  wave_lds_sync();
  u32 beta;
  {
    u32 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = kLBeta[i];
    beta = fsl_from_words(w, k);
  }
#pragma unroll 1
  for (int j = 0; j < GV_QTAB_N / 4; ++j) {
    const int e = 4 * j + (int)row;
    u32 x = lo ? sh.qtab[0][e][L] : 0u, y = lo ? sh.qtab[0][e][9 + L] : 0u;
    if (e != GV_QTAB_N - 1) {                           // the last entry is already on Z_15
      const u32 a = e == 0 ? acc : (lo ? sh.ratio[e - 1][L] : 0u);     // acc_(e+1)
      const u32 a2 = fsl_sqr(a, k);
      const u32 a3 = fsl_mul(a2, a, k);
      x = fsl_mul(x, a2, k);
      y = fsl_mul(y, a3, k);
    }
    const u32 t = fsl_mul(x, beta, k);
    if (lo) {
      sh.qtab[0][e][L] = x; sh.qtab[0][e][9 + L] = y;
      sh.qtab[1][e][L] = t; sh.qtab[1][e][9 + L] = y;
    }
  }
  const u32 zq = fsl_mul(qy << 1, acc, k);              // Z_15 = 2y * prod(ratios)
  if (row == 0u && lo) sh.zq[L] = zq;
}


// Wave 0 of k_verify_lat_sl: key decompression, Q / lambda*Q tables into LDS,
// zq (Z of the table's curve) and the ParsePubKey verdict into LDS.
template <class SH>
GV_DEV void lat_sl_prep(SH& sh, const gvk_lat& b, u32 gi, const fslk& k) {
  fe x8, y8;
  const bool ok = lat_sl_decompress(x8, y8, b, gi, k);
  lat_sl_tables(sh, fsl_from_words(x8.v, k), fsl_from_words(y8.v, k), k);
  if (threadIdx.x == 0) sh.okp = ok ? 1u : 0u;
  LAT_STAMP(2);                                         // trace builds: tables done
}

// GV_LAT_SL_SPLIT: batches of at most this many signatures split the pub33
// ladder's windows over two waves (even windows + G on wave 0, odd windows on
// wave 2; 192-thread blocks): each runs the 125 doublings but only half the
// Q / lambda*Q additions, plus one complete addition through LDS.  Larger
// batches keep one ladder wave (128-thread blocks): past ~1k signatures the
// third wave per block costs more SIMD time than it saves.  0: never split.
#ifndef GV_LAT_SL_SPLIT
#define GV_LAT_SL_SPLIT 512
#endif
__global__ __launch_bounds__(192) void k_verify_lat_sl(const gvk_lat b) {
  __shared__ LatSlShared sh;
  const u32 gi = blockIdx.x;                            // grid = n: every block is live
  const u32 wave = threadIdx.x >> 6;
  if (wave == 0u) LAT_STAMP(0);
  if (wave == 1u) {                                     // the scalar chain, whole wave (own SIMD)
    if (b.msg_len) {                                    // message path: SHA-256 of the sign bytes here
      u32 eh[8];
      sha256_msg_wave(eh, b.msg_blob + b.msg_off[gi], b.msg_len[gi]);
      lat_scalars<true>(sh, 0, true, b.sig64 + (size_t)gi * 64u, nullptr, nullptr, b.C, gi, eh);
    } else {
      lat_scalars<true>(sh, 0, true, b.sig64 + (size_t)gi * 64u, b.dig32 + (size_t)gi * 32u, nullptr, b.C, gi);
    }
    LAT_STAMP(3);                                       // trace builds: scalars done
    __syncthreads();
    __syncthreads();
    return;
  }
  const fslk k = fsl_consts();
  const u32 row = (threadIdx.x >> 4) & 3u, L = k.L;
  const bool lo = L < 9u;
  if (wave == 0u) lat_sl_prep(sh, b, gi, k);
  __syncthreads();                                      // digits (wave 1) + tables, zq (wave 0)
  if (wave == 0u) LAT_STAMP(4);
  const bool ok = sh.okp != 0u;
  const u32 zq = lo ? sh.zq[L] : 0u;
  // ---- ladder: row r accumulates one of the four partial sums (of its wave's windows)
  const bool split = blockDim.x > 128u;
  const int par = split ? (wave == 0u ? 0 : 1) : -1;
  gjsl A;
  A.x = 0u; A.y = 0u; A.z = 0u;
  bool inf = true;
  const u32* gbase = b.gtab + (row == 3u ? (size_t)GV_GTAB_N * 16u : 0u);
#pragma unroll 1
  for (int win = GV_QWIN - 1; win >= 0; --win) {
    // the window's entry is fetched before its doublings: the G rows' global
    // loads (and the LDS reads) complete under the ~4 us of doubling work
    const bool gwin = (win % GV_GSTEP) == 0 && wave == 0u;
    const bool mine = par < 0 || (win & 1) == par;
    const u32 dq = sh.dq[0][win];
    int d;
    if (row < 2u) d = !mine ? 0 : row == 0u ? ((int)(dq << 16) >> 16) : ((int)dq >> 16);
    else d = gwin ? sh.dg[0][win / GV_GSTEP][row - 2u] : 0;
    u32 x = 0u, y = 0u;
    if (d != 0) {
      const u32 e = (u32)((d < 0 ? -d : d) - 1);
      if (row < 2u) {
        x = lo ? sh.qtab[row][e][L] : 0u;
        y = lo ? sh.qtab[row][e][9 + L] : 0u;
      } else {
        const u32* pe = gbase + (size_t)e * 16u;
        x = fsl_load_words(pe, k);
        y = fsl_load_words(pe + 8, k);
      }
    }
    if (win != GV_QWIN - 1) {
#pragma unroll 1
      for (int dd = 0; dd < GV_QW; ++dd) gjsl_double(A, A, k);
    }
    if (d != 0) {
      if (d < 0) y = k.bias - y;
      if (inf) {
        A.x = x; A.y = fsl_norm(y, k); A.z = L == 0u ? 1u : 0u;
        inf = false;
      } else {
        gjsl_add_scaled(A, inf, x, y, A.z, k);
      }
    }
  }
  // ---- combine: Q rows back to the real curve, two rounds across rows,
  // then wave 2's sum into wave 0 through LDS
  if (wave == 0u) LAT_STAMP(5);
  if (row < 2u) A.z = fsl_mul(A.z, zq, k);
#pragma unroll 1
  for (int m = 16; m < 64; m <<= 1) {
    gjsl O;
    O.x = (u32)__shfl_xor((int)A.x, m, 64);
    O.y = (u32)__shfl_xor((int)A.y, m, 64);
    O.z = (u32)__shfl_xor((int)A.z, m, 64);
    const bool oinf = __shfl_xor((int)inf, m, 64) != 0;
    gjsl_add_gej(A, inf, A, inf, O, oinf, k);
  }
  if (wave == 2u && row == 0u) {
    if (lo) { sh.pt[0][L] = A.x; sh.pt[1][L] = A.y; sh.pt[2][L] = A.z; }
    if (L == 0u) sh.pinf = inf ? 1u : 0u;
  }
  __syncthreads();
  if (wave == 2u) return;
  if (split) {
    gjsl O;
    O.x = lo ? sh.pt[0][L] : 0u;
    O.y = lo ? sh.pt[1][L] : 0u;
    O.z = lo ? sh.pt[2][L] : 0u;
    gjsl_add_gej(A, inf, A, inf, O, sh.pinf != 0u, k);
  }
  LAT_STAMP(6);
  // ---- final check (as k_ecmult): x(R) mod n == r, without inversion
  const u32 fl = sh.oks[0];
  bool okv = (fl & 1u) && ok && !inf;
  u32 rw[8], X[8], T[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) rw[i] = sh.r[0][i];
  const u32 zz = fsl_sqr(A.z, k);
  fsl_to_words(X, A.x);
  fsl_to_words(T, fsl_mul(fsl_from_words(rw, k), zz, k));
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) eq &= (X[i] == T[i]);
  if (!eq && (fl & 2u)) {
    u32 rn[8], c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) rn[i] = __builtin_addc(rw[i], kN[i], c, &c);
    fsl_to_words(T, fsl_mul(fsl_from_words(rn, k), zz, k));
    eq = true;
#pragma unroll
    for (int i = 0; i < 8; ++i) eq &= (X[i] == T[i]);
  }
  okv &= eq;
  if (threadIdx.x == 0) {
    if (b.out8) b.out8[gi] = okv ? 1u : 0u;
    else if (okv) atomicOr((unsigned long long*)&b.bits[gi >> 6], 1ull << (gi & 63u));
  }
  LAT_STAMP(7);
}

// ---------------------------------------------------------------------------
// Pub33 small batches, row-parallel (k_verify_lat_sl4): ONE signature per
// 256-thread block, and each ladder wave's four 16-lane rows cooperate on ONE
// accumulator -- the products of a doubling / addition that do not depend on
// each other run in different rows at once and every row gets every row's
// result from three lane swaps (v_permlane16_swap, v_permlane32_swap: VALU,
// no LDS round trip), so a doubling is 3 product rounds instead of 7 serial
// products and an addition 5 instead of 11.
//
// The key's square root is off the critical path: with c = x^3 + 7 the point
// Q' = (c x, c^2) lies on E': Y^2 = X^3 + 7 c^3, the image of Q = (x, y) under
// (x, y) -> (u^2 x, u^3 y) with u = y (u^2 = c), and doubling / addition
// formulas of a = 0 curves never read b: the Q / lambda*Q tables and ladders
// run on Q' as soon as c is known, and a Jacobian (X, Y, Z) of E' is the point
// (X, Y, y Z) of E.  The square root (ParsePubKey's "invalid square root" and
// y's parity) runs on its own wave meanwhile and only y joins at the end.
//
// Waves (one per SIMD), started by LDS flags instead of a block barrier:
//   0: c, tables of Q' (LDS) -> Q ladder, even windows -> the combination
//   1: scalar chain (digits, r) -> lambda*Q ladder, windows 13..25
//   2: (message path: SHA-256 of the sign bytes, handed to wave 1's chain
//      after s^-1) -> Q ladder, odd windows
//   3: square root -> G sum (gtab6: u1 unsplit, 11 signed 24-bit windows, no
//      doublings) -> lambda*Q ladder, windows 0..12 (60 doublings)
// Same checks, group law results (every exceptional case as gjsl_add_scaled /
// gjsl_add_gej, mapped through the isomorphism) and verdict as k_verify_lat_sl.
struct LatSl4Shared {
  static constexpr bool kG5 = false;
  static constexpr bool kG24 = true;
  static constexpr bool kQ6 = false;          // Q digits: 5-bit windows (6-bit: the kn arena)
  u32 qtab[2][GV_QTAB_N][18];               // Q', lambda*Q' entries (effective affine, sliced limbs)
  u32 ratio[GV_QTAB_N - 1][9];
  u32 dq[1][GV_QWIN];
  int dg24[1][GV_K6_GWIN];                  // u1's 24-bit Booth digits
  u32 r[1][8];
  u32 oks[1];
  u32 zq[16];
  u32 okp;                                  // ParsePubKey verdict (wave 3)
  u32 ysl[16];                              // y (wave 3)
  u32 pt[4][3][16];                         // the partial sums of waves 1, 2, 3 and the G sum
  u32 pinf[4];
  u32 gent[GV_K6_GWIN][18];                 // the G entries (x, +-y), sliced
  u32 eh[8];                                // message path: SHA-256 of the sign bytes (wave 2)
  u32 flag_tab, flag_sc, flag_e;            // tables / scalars / digest ready
};


// Every round below is ONE product per lane whose operands (and 64-bit extra)
// the row selects -- never a branch on the row, which would run each row's
// product in turn.
//
// A = 2A, the accumulator replicated in the wave's four rows:
//   round 1: B = Y^2 (row 0), Z3 = Y 2Z (row 1), E = 3X^2 (rows 2, 3)
//   round 2: D = X B (row 0), C = B^2 (row 1), E2 = E^2 (rows 2, 3)
//   round 3: X3 = E^2 - 8D (row 0), Y3 = E (12D - E2) - 8C (rows 1..3)
// (Y3 = E (4D - X3) - 8C with X3 = E^2 - 8D): gjsl_double's values mod p.
GV_DEV void gj4_double(gjsl& A, u32 row, const fslk& k) {
  const rows4 p1 = rows_all(fsl_mul(row >= 2u ? A.x : A.y, row == 0u ? A.y : row == 1u ? A.z << 1 : A.x * 3u, k));
  const u32 B = p1.r[0], Z3 = p1.r[1], E = p1.r[2];
  const rows4 p2 = rows_all(fsl_mul(row == 0u ? A.x : row == 1u ? B : E, row >= 2u ? E : B, k));
  const u32 D = p2.r[0], C = p2.r[1], E2 = p2.r[2];
  const u32 t = (fsl_norm(D * 3u, k) << 2) + k.bias - E2;          // 12D - E^2 < 2^31.6
  const rows4 p3 = rows_all(fsl_mul_plus(E, row == 0u ? E : t, k.big8 - ((u64)(row == 0u ? D : C) << 3), k));
  A.x = p3.r[0];
  A.y = p3.r[1];
  A.z = Z3;
}

// A += (x, y), affine on the curve scaled by A.z (gjsl_add_scaled's formula
// and cases), row-parallel:
//   round 1: z2 = Z1^2 (every row)
//   round 2: H = x z2 - X1 (row 0), z3 = z2 Z1 (rows 1..3)
//   round 3: R = y z3 - Y1 (row 0), H2 = H^2 (row 1), Z3 = Z1 H (row 2), Y1 H (row 3)
//   round 4: H3 = H2 H (row 0), V = X1 H2 (row 1), R2 = R^2 (row 2), Y1 H3 (row 3)
//   X3 = R2 - H3 - 2V (sums only)
//   round 5: Y3 = R (V - X3) - Y1 H3 (every row: nothing to exchange)
GV_DEV void gj4_add(gjsl& A, bool& inf, u32 x, u32 y, u32 row, const fslk& k) {
  const u32 z2 = fsl_sqr(A.z, k);
  const rows4 p2 = rows_all(fsl_mul_plus(row == 0u ? x : z2, row == 0u ? z2 : A.z,
                                         row == 0u ? (u64)(k.bias - A.x) : 0ull, k));
  const u32 h = p2.r[0], z3 = p2.r[1];
  const rows4 p3 = rows_all(fsl_mul_plus(row == 0u ? y : row == 1u ? h : row == 2u ? A.z : A.y, row == 0u ? z3 : h,
                                         row == 0u ? (u64)(k.bias - A.y) : 0ull, k));
  const u32 rr = p3.r[0];
  if (fsl_is_zero(h)) {                                  // the same answer in every row
    if (fsl_is_zero(rr)) gj4_double(A, row, k);          // A == entry: 2A
    else inf = true;                                     // A == -entry
    return;
  }
  const u32 h2 = p3.r[1], zn = p3.r[2], y1h = p3.r[3];
  const rows4 p4 = rows_all(fsl_mul(row == 0u ? h2 : row == 1u ? A.x : row == 2u ? rr : y1h,
                                    row == 0u ? h : row == 2u ? rr : h2, k));
  const u32 h3 = p4.r[0], v = p4.r[1], r2 = p4.r[2], y1h3 = p4.r[3];
  const u32 x3 = fsl_norm(r2 + 3u * k.bias - h3 - (v << 1), k);   // < 2^31.9 before the carry pass
  A.y = fsl_mul_plus(rr, v + k.bias - x3, (u64)(k.bias - y1h3), k);
  A.x = x3;
  A.z = zn;
}

// A += O, two Jacobian points of the real curve (gjsl_add_gej's formula and
// cases: either infinite -> the other; A == O -> 2A; A == -O -> infinity):
//   round 1: Z1^2 (row 0), Z2^2 (row 1), Z1 Z2 (rows 2, 3)
//   round 2: U1 = X1 Z2^2 (row 0), U2 = X2 Z1^2 (row 1), Z2^3 (row 2), Z1^3 (row 3)
//   round 3: S1 = Y1 Z2^3 (row 0), S2 = Y2 Z1^3 (row 1), Z3 = Z1 Z2 H (row 2), H2 = H^2 (row 3)
//   round 4: R2 = R^2 (row 0), H3 = H2 H (row 1), V = U1 H2 (rows 2, 3)
//   X3 = R2 - H3 - 2V (sums only)
//   round 5: Y3 = R (V - X3) - S1 H3 (every row)
GV_DEV void gj4_add_gej(gjsl& A, bool& inf, const gjsl& O, bool oinf, u32 row, const fslk& k) {
  if (inf || oinf) {
    if (inf) A = O;
    inf = inf && oinf;
    return;
  }
  const rows4 p1 = rows_all(fsl_mul(row == 1u ? O.z : A.z, row == 0u ? A.z : O.z, k));
  const u32 z11 = p1.r[0], z22 = p1.r[1], z12 = p1.r[2];
  const rows4 p2 = rows_all(fsl_mul(row == 0u ? A.x : row == 1u ? O.x : row == 2u ? O.z : A.z,
                                    row == 0u || row == 2u ? z22 : z11, k));
  const u32 u1 = p2.r[0], u2 = p2.r[1], z23 = p2.r[2], z13 = p2.r[3];
  const u32 h = fsl_sub(u2, u1, k);
  const rows4 p3 = rows_all(fsl_mul(row == 0u ? A.y : row == 1u ? O.y : row == 2u ? z12 : h,
                                    row == 0u ? z23 : row == 1u ? z13 : h, k));
  const u32 s1 = p3.r[0], s2 = p3.r[1];
  const u32 rr = fsl_sub(s2, s1, k);
  if (fsl_is_zero(h)) {
    if (fsl_is_zero(rr)) gj4_double(A, row, k);
    else inf = true;
    return;
  }
  const u32 zn = p3.r[2], h2 = p3.r[3];
  const rows4 p4 = rows_all(fsl_mul(row == 0u ? rr : row == 1u ? h2 : u1, row == 0u ? rr : row == 1u ? h : h2, k));
  const u32 r2 = p4.r[0], h3 = p4.r[1], v = p4.r[2];
  const u32 x3 = fsl_norm(r2 + 3u * k.bias - h3 - (v << 1), k);
  A.y = fsl_mul2(rr, v + k.bias - x3, k.bias - s1, h3, k);
  A.x = x3;
  A.z = zn;
}

// A += the affine point (x, y) (sliced limbs, y < 2^30.1); A may be infinity
GV_DEV void gj4_add_affine(gjsl& A, bool& inf, u32 x, u32 y, u32 row, const fslk& k) {
  if (inf) {
    A.x = x; A.y = fsl_norm(y, k); A.z = k.L == 0u ? 1u : 0u;
    inf = false;
  } else {
    gj4_add(A, inf, x, y, row, k);
  }
}

__global__ __launch_bounds__(256) void k_verify_lat_sl4(const gvk_lat b) {
  __shared__ LatSl4Shared sh;
  const u32 gi = blockIdx.x;                            // grid = n: every block is live
  const u32 wave = threadIdx.x >> 6;
  const fslk k = fsl_consts();
  const u32 row = (threadIdx.x >> 4) & 3u, L = k.L;
  const bool lo = L < 9u;
  if (threadIdx.x == 0) { sh.flag_tab = 0u; sh.flag_sc = 0u; sh.flag_e = 0u; }
  __syncthreads();
  if (wave == 0u) LAT_STAMP(0);
  gjsl A;
  A.x = 0u; A.y = 0u; A.z = 0u;
  bool inf = true;
  if (wave == 0u) {                                     // tables of Q' = (c x, c^2)
    const uint8_t* p = b.pub33 + (size_t)gi * 33u;
    u32 xw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) xw[i] = be32(p + 1 + 4 * (7 - i));
    const u32 xs = fsl_from_words(xw, k);
    const u32 c = fsl_mul(fsl_sqr(xs, k), xs, k) + (L == 0u ? 7u : 0u);
    lat_sl_tables(sh, fsl_mul(c, xs, k), fsl_sqr(c, k), k);
    LAT_STAMP(2);                                       // trace builds: tables done
    lds_flag_set(&sh.flag_tab);
  } else if (wave == 1u) {                              // the scalar chain
    if (b.msg_len) {                                    // e from wave 2's hash, first needed after s^-1
      lat_scalars_e<true>(sh, 0, true, b.sig64 + (size_t)gi * 64u, [&](u32 e[8]) {
        lds_flag_wait(&sh.flag_e);
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = sh.eh[7 - i];
      });
    } else {
      lat_scalars<true>(sh, 0, true, b.sig64 + (size_t)gi * 64u, b.dig32 + (size_t)gi * 32u, nullptr, b.C, gi);
    }
    LAT_STAMP(3);                                       // trace builds: scalars done
    lds_flag_set(&sh.flag_sc);
  } else if (wave == 2u) {                              // message path: the hash, beside s^-1
    if (b.msg_len) {
      u32 eh[8];
      sha256_msg_wave(eh, b.msg_blob + b.msg_off[gi], b.msg_len[gi]);
      if (threadIdx.x == 128u) {
#pragma unroll
        for (int i = 0; i < 8; ++i) sh.eh[i] = eh[i];
      }
      lds_flag_set(&sh.flag_e);
    }
  } else if (wave == 3u) {                              // ParsePubKey's square root, then G
    fe x8, y8;
    const bool ok = lat_sl_decompress(x8, y8, b, gi, k);
    const u32 y = fsl_from_words(y8.v, k);
    if (row == 0u && lo) sh.ysl[L] = y;
    if (threadIdx.x == 192u) sh.okp = ok ? 1u : 0u;
    lds_flag_wait(&sh.flag_sc);
    // G = sum of d_j (2^(24 j) G): every entry's loads in flight at once,
    // parked in LDS (row j & 3 stores entry j)
#pragma unroll
    for (int j = 0; j < GV_K6_GWIN; ++j) {
      const int d = sh.dg24[0][j];
      const u32 e = d == 0 ? 0u : (u32)((d < 0 ? -d : d) - 1);
      const u32* pe = b.gtab6 + ((size_t)j * GV_K6_GTAB_N + e) * 16u;
      const u32 x = fsl_load_words(pe, k), yv = fsl_load_words(pe + 8, k);
      if (row == (u32)(j & 3) && lo) { sh.gent[j][L] = x; sh.gent[j][9 + L] = d < 0 ? k.bias - yv : yv; }
    }
    wave_lds_sync();
#pragma unroll 1
    for (int j = 0; j < GV_K6_GWIN; ++j) {
      if (sh.dg24[0][j] == 0) continue;
      gj4_add_affine(A, inf, lo ? sh.gent[j][L] : 0u, lo ? sh.gent[j][9 + L] : 0u, row, k);
    }
    if (row == 0u) {
      if (lo) { sh.pt[3][0][L] = A.x; sh.pt[3][1][L] = A.y; sh.pt[3][2][L] = A.z; }
      if (L == 0u) sh.pinf[3] = inf ? 1u : 0u;
    }
    LAT_STAMP(7);                                       // trace builds: G sum done
    A.x = 0u; A.y = 0u; A.z = 0u;
    inf = true;
  }
  lds_flag_wait(&sh.flag_tab);
  lds_flag_wait(&sh.flag_sc);
  if (wave == 0u) LAT_STAMP(4);
  {
    // wave 0: Q even windows, 2: Q odd, 1: lambda*Q windows 13..25, 3: lambda*Q windows 0..12
    const int tab = (wave == 0u || wave == 2u) ? 0 : 1;
    const int top = wave == 3u ? GV_QWIN / 2 - 1 : GV_QWIN - 1;
#pragma unroll 1
    for (int win = top; win >= 0; --win) {
      if (win != top && !inf) {
#pragma unroll 1
        for (int dd = 0; dd < GV_QW; ++dd) gj4_double(A, row, k);
      }
      const bool mine = wave == 0u ? (win & 1) == 0 : wave == 2u ? (win & 1) == 1
                      : wave == 1u ? win >= GV_QWIN / 2 : true;
      if (!mine) continue;
      const u32 dq = sh.dq[0][win];
      const int d = tab == 0 ? ((int)(dq << 16) >> 16) : ((int)dq >> 16);
      if (d == 0) continue;
      const u32 e = (u32)((d < 0 ? -d : d) - 1);
      const u32 x = lo ? sh.qtab[tab][e][L] : 0u;
      const u32 y = lo ? sh.qtab[tab][e][9 + L] : 0u;
      gj4_add_affine(A, inf, x, d < 0 ? k.bias - y : y, row, k);
    }
  }
  if (wave == 0u) LAT_STAMP(5);
  if (wave != 0u && row == 0u) {                        // partial sums into LDS, wave 0 adds them
    if (lo) { sh.pt[wave - 1][0][L] = A.x; sh.pt[wave - 1][1][L] = A.y; sh.pt[wave - 1][2][L] = A.z; }
    if (L == 0u) sh.pinf[wave - 1] = inf ? 1u : 0u;
  }
  __syncthreads();
  if (wave != 0u) return;
  // the Q' partial sums (the tables' curve), then back to E: Z * zq * y
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    if (j == 3 && !inf) A.z = fsl_mul(A.z, fsl_mul(lo ? sh.zq[L] : 0u, lo ? sh.ysl[L] : 0u, k), k);
    gjsl O;
    O.x = lo ? sh.pt[j][0][L] : 0u;
    O.y = lo ? sh.pt[j][1][L] : 0u;
    O.z = lo ? sh.pt[j][2][L] : 0u;
    gj4_add_gej(A, inf, O, sh.pinf[j] != 0u, row, k);
  }
  LAT_STAMP(6);
  // ---- final check (as k_verify_lat_sl): x(R) mod n == r, without inversion
  const bool ok = sh.okp != 0u;
  const u32 fl = sh.oks[0];
  bool okv = (fl & 1u) && ok && !inf;
  u32 rw[8], X[8], T[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) rw[i] = sh.r[0][i];
  const u32 zz = fsl_sqr(A.z, k);
  fsl_to_words(X, A.x);
  fsl_to_words(T, fsl_mul(fsl_from_words(rw, k), zz, k));
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) eq &= (X[i] == T[i]);
  if (!eq && (fl & 2u)) {
    u32 rn[8], c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) rn[i] = __builtin_addc(rw[i], kN[i], c, &c);
    fsl_to_words(T, fsl_mul(fsl_from_words(rn, k), zz, k));
    eq = true;
#pragma unroll
    for (int i = 0; i < 8; ++i) eq &= (X[i] == T[i]);
  }
  okv &= eq;
  if (threadIdx.x == 0) {
    if (b.out8) b.out8[gi] = okv ? 1u : 0u;
    else if (okv) atomicOr((unsigned long long*)&b.bits[gi >> 6], 1ull << (gi & 63u));
  }
}

// ---------------------------------------------------------------------------
// Keyed small batches on the limb-sliced layer: ONE signature per 256-thread
// block.  Lane 0 runs the scalar chain; then wave g (window group g of
// k_verify_lat16) row r accumulates part r of {k1q Q, k2q lambda Q, k1g G,
// k2g lambda G} over that group's <= 7 windows (<= 30 doublings) against the
// arena group table (Q) or glat (G), one element per 16-lane row; two
// cross-row rounds give each wave its group sum, two more (through LDS, in
// wave 0) the whole sum, and wave 0 runs the final check.
struct Lat16SlShared {
  static constexpr bool kG5 = true;
  static constexpr bool kG24 = false;
  static constexpr bool kQ6 = false;          // Q digits: 5-bit windows (6-bit: the kn arena)
  u32 eh[8];                                // message path: the SHA-256 state of the sign bytes (wave 1)
  u32 dq[1][GV_QWIN];
  u32 dg5[1][GV_QWIN];
  u32 r[1][8];
  u32 oks[1];
  u32 pt[GV_LGRP][3][16];                   // group sums, sliced (x, y, z rows)
  u32 pinf[GV_LGRP];
};

__global__ __launch_bounds__(256) void k_verify_lat16_sl(const gvk_lat b) {
  __shared__ Lat16SlShared sh;
  const u32 gi = blockIdx.x;                            // grid = n: every block is live
  u32 sl = b.kslot[gi];
  bool kok = sl < b.kcount;
  if (!kok) sl = 0;                                     // the arena always holds slot 0's memory
  kok = kok && b.kok[sl] != 0u;
  if (b.msg_len) {
    // message path: wave 1 hashes the sign bytes while wave 0 runs the
    // scalar chain up to s^-1; one extra barrier hands the digest over
    if (threadIdx.x < 64) {
      lat_scalars_e<true>(sh, 0, true, b.sig64 + (size_t)gi * 64u, [&](u32 e[8]) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = sh.eh[7 - i];
      });
    } else {
      if (threadIdx.x < 128) {
        u32 eh[8];
        sha256_msg_wave(eh, b.msg_blob + b.msg_off[gi], b.msg_len[gi]);
        if (threadIdx.x == 64) {
#pragma unroll
          for (int i = 0; i < 8; ++i) sh.eh[i] = eh[i];
        }
      }
      __syncthreads();
    }
  } else if (threadIdx.x < 64) {                        // wave 0: the scalar chain, whole wave
    lat_scalars<true>(sh, 0, true, b.sig64 + (size_t)gi * 64u, b.dig32 + (size_t)gi * 32u, nullptr, b.C, gi);
  }
  __syncthreads();
  const fslk k = fsl_consts();
  const u32 L = k.L, part = (threadIdx.x >> 4) & 3u, grp = threadIdx.x >> 6;
  const bool lo = L < 9u;
  const int w_lo = kL16Win[grp], w_hi = kL16Win[grp + 1] - 1;
  u32 beta;
  {
    u32 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = kLBeta[i];
    beta = fsl_from_words(w, k);
  }
  const u32* qrow = grp == 0u ? b.kqt + (size_t)sl * GV_QTAB_N * GV_QENT_WORDS
                              : b.kqt2 + ((size_t)sl * GV_KEY2_TABLES + (grp - 1u)) * GV_QTAB_N * GV_QENT_WORDS;
  const u32* grow = b.glat + (size_t)(grp * 2u + (part & 1u)) * GV_QTAB_N * 16u;
  gjsl A;
  A.x = 0u; A.y = 0u; A.z = 0u;
  bool inf = true;
#pragma unroll 1
  for (int win = w_hi; win >= w_lo; --win) {
    // the window's entry (HBM: key arena / glat) is fetched before its
    // doublings, so the load latency hides under them
    const u32 dw = part < 2u ? sh.dq[0][win] : sh.dg5[0][win];
    const int d = (part & 1u) == 0u ? ((int)(dw << 16) >> 16) : ((int)dw >> 16);
    u32 x = 0u, y = 0u;
    if (d != 0) {
      const u32 e = (u32)((d < 0 ? -d : d) - 1);
      if (part < 2u) {                                  // Q / lambda Q: arena row, 29-bit limbs
        const u32* pe = qrow + (size_t)e * GV_QENT_WORDS;
        x = lo ? pe[L] : 0u;
        y = lo ? pe[9 + L] : 0u;
      } else {                                          // G / lambda G: affine words
        const u32* pe = grow + (size_t)e * 16u;
        x = fsl_load_words(pe, k);
        y = fsl_load_words(pe + 8, k);
      }
    }
    if (win != w_hi) {
#pragma unroll 1
      for (int dd = 0; dd < GV_QW; ++dd) gjsl_double(A, A, k);
    }
    if (d != 0) {
      if (part == 1u) x = fsl_mul(x, beta, k);          // lambda Q = (beta x, y), same Z
      if (d < 0) y = k.bias - y;
      if (inf) {
        A.x = x; A.y = fsl_norm(y, k); A.z = L == 0u ? 1u : 0u;
        inf = false;
      } else {
        gjsl_add_scaled(A, inf, x, y, A.z, k);
      }
    }
  }
  if (part < 2u) {                                      // Q parts: back to the real curve
    const u32* zrow = grp == 0u ? b.kzq : b.kzq2 + (size_t)(grp - 1u) * 8u * b.kC;
    u32 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = zrow[(size_t)i * b.kC + sl];
    A.z = fsl_mul(A.z, fsl_from_words(w, k), k);
  }
#pragma unroll 1
  for (int m = 16; m < 64; m <<= 1) {                   // the group's four parts
    gjsl O;
    O.x = (u32)__shfl_xor((int)A.x, m, 64);
    O.y = (u32)__shfl_xor((int)A.y, m, 64);
    O.z = (u32)__shfl_xor((int)A.z, m, 64);
    const bool oinf = __shfl_xor((int)inf, m, 64) != 0;
    gjsl_add_gej(A, inf, A, inf, O, oinf, k);
  }
  if (part == 0u) {
    if (lo) { sh.pt[grp][0][L] = A.x; sh.pt[grp][1][L] = A.y; sh.pt[grp][2][L] = A.z; }
    if (L == 0u) sh.pinf[grp] = inf ? 1u : 0u;
  }
  __syncthreads();
  if (grp != 0u) return;
  A.x = lo ? sh.pt[part][0][L] : 0u;                    // wave 0, row r: group r's sum
  A.y = lo ? sh.pt[part][1][L] : 0u;
  A.z = lo ? sh.pt[part][2][L] : 0u;
  inf = sh.pinf[part] != 0u;
#pragma unroll 1
  for (int m = 16; m < 64; m <<= 1) {
    gjsl O;
    O.x = (u32)__shfl_xor((int)A.x, m, 64);
    O.y = (u32)__shfl_xor((int)A.y, m, 64);
    O.z = (u32)__shfl_xor((int)A.z, m, 64);
    const bool oinf = __shfl_xor((int)inf, m, 64) != 0;
    gjsl_add_gej(A, inf, A, inf, O, oinf, k);
  }
  const u32 fl = sh.oks[0];
  bool okv = (fl & 1u) && kok && !inf;
  u32 rw[8], X[8], T[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) rw[i] = sh.r[0][i];
  const u32 zz = fsl_sqr(A.z, k);
  fsl_to_words(X, A.x);
  fsl_to_words(T, fsl_mul(fsl_from_words(rw, k), zz, k));
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) eq &= (X[i] == T[i]);
  if (!eq && (fl & 2u)) {
    u32 rn[8], c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) rn[i] = __builtin_addc(rw[i], kN[i], c, &c);
    fsl_to_words(T, fsl_mul(fsl_from_words(rn, k), zz, k));
    eq = true;
#pragma unroll
    for (int i = 0; i < 8; ++i) eq &= (X[i] == T[i]);
  }
  okv &= eq;
  if (threadIdx.x == 0) {
    if (b.out8) b.out8[gi] = okv ? 1u : 0u;
    else if (okv) atomicOr((unsigned long long*)&b.bits[gi >> 6], 1ull << (gi & 63u));
  }
}

// ---------------------------------------------------------------------------
// Keyed small batches on the resident arena's kn tables (k_verify_lat16_kn):
// the slot's 11 group tables of 32 entries (2^(12 g) Q, g < 11, on one Z,
// 6-bit Booth windows: window 2g + p at position p of group g) need only 6
// doublings, and G comes from the 24-bit tables (u1 unsplit, 11 windows, no
// doubling at all).  One signature per 256-thread block, 16 rows: row g < 11
// adds group g's Q and lambda*Q entries of its two positions around the 6
// doublings and lifts its sum by the tables' Z; rows 12..15 (wave 3) add the
// G windows j == row - 12 (mod 4); row 11 has nothing to add.  The 16 sums
// are joined four per wave with the row-parallel complete addition
// (gj4_add_gej), then by wave 0.  Same verdicts as k_verify_lat16_sl.
struct Lat16KnShared {
  static constexpr bool kG5 = false;
  static constexpr bool kG24 = true;
  static constexpr bool kQ6 = true;
  u32 eh[8];                                // message path: the SHA-256 state of the sign bytes (wave 1)
  u32 dq[1][GV_QWIN];                       // GV_K6_QWIN used
  int dg24[1][GV_K6_GWIN];
  u32 r[1][8];
  u32 oks[1];
  u32 pt[16][3][16];                        // the rows' sums, sliced
  u32 pinf[16];
  u32 pw[4][3][16];                         // the waves' sums
  u32 pwinf[4];
};
static_assert(GV_K6_QWIN == 2 * GV_KN_ARENA_NG && GV_KN_ARENA_NG <= 12 && GV_K6_GWIN <= 12, "kn rows");

__global__ __launch_bounds__(256) void k_verify_lat16_kn(const gvk_lat b) {
  __shared__ Lat16KnShared sh;
  const u32 gi = blockIdx.x;                            // grid = n: every block is live
  u32 sl = b.kslot[gi];
  bool kok = sl < b.kcount;
  if (!kok) sl = 0;                                     // the arena always holds slot 0's memory
  kok = kok && b.kok[sl] != 0u;
  if (b.msg_len) {
    if (threadIdx.x < 64) {
      lat_scalars_e<true>(sh, 0, true, b.sig64 + (size_t)gi * 64u, [&](u32 e[8]) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = sh.eh[7 - i];
      });
    } else {
      if (threadIdx.x < 128) {
        u32 eh[8];
        sha256_msg_wave(eh, b.msg_blob + b.msg_off[gi], b.msg_len[gi]);
        if (threadIdx.x == 64) {
#pragma unroll
          for (int i = 0; i < 8; ++i) sh.eh[i] = eh[i];
        }
      }
      __syncthreads();
    }
  } else if (threadIdx.x < 64) {
    lat_scalars<true>(sh, 0, true, b.sig64 + (size_t)gi * 64u, b.dig32 + (size_t)gi * 32u, nullptr, b.C, gi);
  }
  __syncthreads();
  const fslk k = fsl_consts();
  const u32 L = k.L, r16 = threadIdx.x >> 4, wave = threadIdx.x >> 6, row = r16 & 3u;
  const bool lo = L < 9u;
  gjsl A;
  A.x = 0u; A.y = 0u; A.z = 0u;
  bool inf = true;
  if (wave < 3u) {                                      // rows 0..11: Q groups (row 11: none)
    const u32 g = r16;
    u32 beta;
    {
      u32 w[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) w[i] = kLBeta[i];
      beta = fsl_from_words(w, k);
    }
    const u32* tab = g == 0u ? b.kqt + (size_t)sl * GV_K6_KEY_WORDS
                             : b.kqt2 + ((size_t)sl * (GV_KN_ARENA_NG - 1) + (g - 1u)) * GV_K6_KEY_WORDS;
#pragma unroll 1
    for (int p = 1; p >= 0; --p) {
      if (p == 0 && !inf) {
#pragma unroll 1
        for (int dd = 0; dd < GV_K6_QW; ++dd) gjsl_double(A, A, k);
      }
      const u32 dq = g < GV_KN_ARENA_NG ? sh.dq[0][2u * g + (u32)p] : 0u;
#pragma unroll 1
      for (int t = 0; t < 2; ++t) {
        const int d = t == 0 ? ((int)(dq << 16) >> 16) : ((int)dq >> 16);
        if (d == 0) continue;
        const u32* pe = tab + (size_t)((d < 0 ? -d : d) - 1) * GV_QENT_WORDS;
        u32 x = lo ? pe[L] : 0u;
        u32 y = lo ? pe[9 + L] : 0u;
        if (t == 1) x = fsl_mul(x, beta, k);            // lambda Q = (beta x, y), same Z
        if (d < 0) y = k.bias - y;
        if (inf) {
          A.x = x; A.y = fsl_norm(y, k); A.z = L == 0u ? 1u : 0u;
          inf = false;
        } else {
          gjsl_add_scaled(A, inf, x, y, A.z, k);
        }
      }
    }
    {                                                   // back to the real curve: Z * (the tables' Z)
      u32 w[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) w[i] = b.kzq[(size_t)i * b.kC + sl];
      A.z = fsl_mul(A.z, fsl_from_words(w, k), k);
    }
  } else {                                              // rows 12..15: G windows j = row (mod 4)
#pragma unroll 1
    for (u32 j = row; j < GV_K6_GWIN; j += 4u) {
      const int d = sh.dg24[0][j];
      if (d == 0) continue;
      const u32* pe = b.gtab6 + ((size_t)j * GV_K6_GTAB_N + (u32)((d < 0 ? -d : d) - 1)) * 16u;
      const u32 x = fsl_load_words(pe, k);
      u32 y = fsl_load_words(pe + 8, k);
      if (d < 0) y = k.bias - y;
      if (inf) {
        A.x = x; A.y = fsl_norm(y, k); A.z = L == 0u ? 1u : 0u;
        inf = false;
      } else {
        gjsl_add_scaled(A, inf, x, y, A.z, k);
      }
    }
  }
  if (lo) { sh.pt[r16][0][L] = A.x; sh.pt[r16][1][L] = A.y; sh.pt[r16][2][L] = A.z; }
  if (L == 0u) sh.pinf[r16] = inf ? 1u : 0u;
  __syncthreads();
  // each wave: its four rows' sums, replicated over its rows, row-parallel additions
  {
    const u32 r0 = wave * 4u;
    A.x = lo ? sh.pt[r0][0][L] : 0u; A.y = lo ? sh.pt[r0][1][L] : 0u; A.z = lo ? sh.pt[r0][2][L] : 0u;
    inf = sh.pinf[r0] != 0u;
#pragma unroll 1
    for (u32 j = 1; j < 4u; ++j) {
      gjsl O;
      O.x = lo ? sh.pt[r0 + j][0][L] : 0u; O.y = lo ? sh.pt[r0 + j][1][L] : 0u; O.z = lo ? sh.pt[r0 + j][2][L] : 0u;
      gj4_add_gej(A, inf, O, sh.pinf[r0 + j] != 0u, row, k);
    }
    if (row == 0u) {
      if (lo) { sh.pw[wave][0][L] = A.x; sh.pw[wave][1][L] = A.y; sh.pw[wave][2][L] = A.z; }
      if (L == 0u) sh.pwinf[wave] = inf ? 1u : 0u;
    }
  }
  __syncthreads();
  if (wave != 0u) return;
#pragma unroll 1
  for (u32 j = 1; j < 4u; ++j) {
    gjsl O;
    O.x = lo ? sh.pw[j][0][L] : 0u; O.y = lo ? sh.pw[j][1][L] : 0u; O.z = lo ? sh.pw[j][2][L] : 0u;
    gj4_add_gej(A, inf, O, sh.pwinf[j] != 0u, row, k);
  }
  const u32 fl = sh.oks[0];
  bool okv = (fl & 1u) && kok && !inf;
  u32 rw[8], X[8], T[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) rw[i] = sh.r[0][i];
  const u32 zz = fsl_sqr(A.z, k);
  fsl_to_words(X, A.x);
  fsl_to_words(T, fsl_mul(fsl_from_words(rw, k), zz, k));
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) eq &= (X[i] == T[i]);
  if (!eq && (fl & 2u)) {
    u32 rn[8], c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) rn[i] = __builtin_addc(rw[i], kN[i], c, &c);
    fsl_to_words(T, fsl_mul(fsl_from_words(rn, k), zz, k));
    eq = true;
#pragma unroll
    for (int i = 0; i < 8; ++i) eq &= (X[i] == T[i]);
  }
  okv &= eq;
  if (threadIdx.x == 0) {
    if (b.out8) b.out8[gi] = okv ? 1u : 0u;
    else if (okv) atomicOr((unsigned long long*)&b.bits[gi >> 6], 1ull << (gi & 63u));
  }
}

// Keyed small batches on the resident arena's wide-window tables
// (k_verify_lat16_kw, round 6): the slot's GV_KW_NG1 group tables of
// 2^(QW-1) entries (one QW-bit Booth window per group and GLV half, 64-B
// canonical entries on one Z) need no doubling at all.  One signature per
// 256-thread block, 16 rows: row g < GV_KW_NG1 adds group g's Q and lambda*Q
// entries and lifts its sum by the tables' Z; rows 12..15 (wave 3) add the G
// windows j == row - 12 (mod 4) from the 24-bit tables.  The 16 sums are
// joined as in k_verify_lat16_kn.  Same verdicts as k_verify_lat16_sl.
struct Lat16KwShared {
  static constexpr bool kG5 = false;
  static constexpr bool kG24 = true;
  static constexpr bool kQ6 = false;
  static constexpr bool kKW = true;         // Q digits: GV_KW_QW-bit windows (lat_q_width)
  u32 eh[8];
  u32 dq[1][GV_QWIN];                       // GV_KW_QWIN used
  int dg24[1][GV_K6_GWIN];
  u32 r[1][8];
  u32 oks[1];
  u32 pt[16][3][16];
  u32 pinf[16];
  u32 pw[4][3][16];
  u32 pwinf[4];
};
static_assert(GV_KW_NG1 == GV_KW_QWIN && GV_KW_NG1 <= 12 && GV_KW_QWIN <= GV_QWIN && GV_K6_GWIN <= 12 &&
                  GV_KW_ENT_WORDS == 16,
              "kw rows: one window per group in rows 0..11, 64-B canonical entries");

__global__ __launch_bounds__(256) void k_verify_lat16_kw(const gvk_lat b) {
  __shared__ Lat16KwShared sh;
  const u32 gi = blockIdx.x;                            // grid = n: every block is live
  u32 sl = b.kslot[gi];
  bool kok = sl < b.kcount;
  if (!kok) sl = 0;                                     // the arena always holds slot 0's memory
  kok = kok && b.kok[sl] != 0u;
  if (b.msg_len) {
    if (threadIdx.x < 64) {
      lat_scalars_e<true>(sh, 0, true, b.sig64 + (size_t)gi * 64u, [&](u32 e[8]) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = sh.eh[7 - i];
      });
    } else {
      if (threadIdx.x < 128) {
        u32 eh[8];
        sha256_msg_wave(eh, b.msg_blob + b.msg_off[gi], b.msg_len[gi]);
        if (threadIdx.x == 64) {
#pragma unroll
          for (int i = 0; i < 8; ++i) sh.eh[i] = eh[i];
        }
      }
      __syncthreads();
    }
  } else if (threadIdx.x < 64) {
    lat_scalars<true>(sh, 0, true, b.sig64 + (size_t)gi * 64u, b.dig32 + (size_t)gi * 32u, nullptr, b.C, gi);
  }
  __syncthreads();
  const fslk k = fsl_consts();
  const u32 L = k.L, r16 = threadIdx.x >> 4, wave = threadIdx.x >> 6, row = r16 & 3u;
  const bool lo = L < 9u;
  gjsl A;
  A.x = 0u; A.y = 0u; A.z = 0u;
  bool inf = true;
  if (wave < 3u) {                                      // rows 0..11: Q groups
    const u32 g = r16;
    if (g < (u32)GV_KW_NG1) {
      u32 beta;
      {
        u32 w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = kLBeta[i];
        beta = fsl_from_words(w, k);
      }
      const u32* tab = g == 0u ? b.kqt + (size_t)sl * GV_KW_KEY_WORDS
                               : b.kqt2 + ((size_t)sl * (GV_KW_NG1 - 1) + (g - 1u)) * GV_KW_KEY_WORDS;
      const u32 dq = sh.dq[0][g];
#pragma unroll 1
      for (int t = 0; t < 2; ++t) {
        const int d = t == 0 ? ((int)(dq << 16) >> 16) : ((int)dq >> 16);
        if (d == 0) continue;
        const u32* pe = tab + (size_t)((d < 0 ? -d : d) - 1) * GV_KW_ENT_WORDS;
        u32 x = fsl_load_words(pe, k);
        u32 y = fsl_load_words(pe + 8, k);
        if (t == 1) x = fsl_mul(x, beta, k);            // lambda Q = (beta x, y), same Z
        if (d < 0) y = k.bias - y;
        if (inf) {
          A.x = x; A.y = fsl_norm(y, k); A.z = L == 0u ? 1u : 0u;
          inf = false;
        } else {
          gjsl_add_scaled(A, inf, x, y, A.z, k);
        }
      }
      {                                                 // back to the real curve: Z * (the tables' Z)
        u32 w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = b.kzq[(size_t)i * b.kC + sl];
        A.z = fsl_mul(A.z, fsl_from_words(w, k), k);
      }
    }
  } else {                                              // rows 12..15: G windows j = row (mod 4)
#pragma unroll 1
    for (u32 j = row; j < GV_K6_GWIN; j += 4u) {
      const int d = sh.dg24[0][j];
      if (d == 0) continue;
      const u32* pe = b.gtab6 + ((size_t)j * GV_K6_GTAB_N + (u32)((d < 0 ? -d : d) - 1)) * 16u;
      const u32 x = fsl_load_words(pe, k);
      u32 y = fsl_load_words(pe + 8, k);
      if (d < 0) y = k.bias - y;
      if (inf) {
        A.x = x; A.y = fsl_norm(y, k); A.z = L == 0u ? 1u : 0u;
        inf = false;
      } else {
        gjsl_add_scaled(A, inf, x, y, A.z, k);
      }
    }
  }
  if (lo) { sh.pt[r16][0][L] = A.x; sh.pt[r16][1][L] = A.y; sh.pt[r16][2][L] = A.z; }
  if (L == 0u) sh.pinf[r16] = inf ? 1u : 0u;
  __syncthreads();
  {
    const u32 r0 = wave * 4u;
    A.x = lo ? sh.pt[r0][0][L] : 0u; A.y = lo ? sh.pt[r0][1][L] : 0u; A.z = lo ? sh.pt[r0][2][L] : 0u;
    inf = sh.pinf[r0] != 0u;
#pragma unroll 1
    for (u32 j = 1; j < 4u; ++j) {
      gjsl O;
      O.x = lo ? sh.pt[r0 + j][0][L] : 0u; O.y = lo ? sh.pt[r0 + j][1][L] : 0u; O.z = lo ? sh.pt[r0 + j][2][L] : 0u;
      gj4_add_gej(A, inf, O, sh.pinf[r0 + j] != 0u, row, k);
    }
    if (row == 0u) {
      if (lo) { sh.pw[wave][0][L] = A.x; sh.pw[wave][1][L] = A.y; sh.pw[wave][2][L] = A.z; }
      if (L == 0u) sh.pwinf[wave] = inf ? 1u : 0u;
    }
  }
  __syncthreads();
  if (wave != 0u) return;
#pragma unroll 1
  for (u32 j = 1; j < 4u; ++j) {
    gjsl O;
    O.x = lo ? sh.pw[j][0][L] : 0u; O.y = lo ? sh.pw[j][1][L] : 0u; O.z = lo ? sh.pw[j][2][L] : 0u;
    gj4_add_gej(A, inf, O, sh.pwinf[j] != 0u, row, k);
  }
  const u32 fl = sh.oks[0];
  bool okv = (fl & 1u) && kok && !inf;
  u32 rw[8], X[8], T[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) rw[i] = sh.r[0][i];
  const u32 zz = fsl_sqr(A.z, k);
  fsl_to_words(X, A.x);
  fsl_to_words(T, fsl_mul(fsl_from_words(rw, k), zz, k));
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) eq &= (X[i] == T[i]);
  if (!eq && (fl & 2u)) {
    u32 rn[8], c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) rn[i] = __builtin_addc(rw[i], kN[i], c, &c);
    fsl_to_words(T, fsl_mul(fsl_from_words(rn, k), zz, k));
    eq = true;
#pragma unroll
    for (int i = 0; i < 8; ++i) eq &= (X[i] == T[i]);
  }
  okv &= eq;
  if (threadIdx.x == 0) {
    if (b.out8) b.out8[gi] = okv ? 1u : 0u;
    else if (okv) atomicOr((unsigned long long*)&b.bits[gi >> 6], 1ull << (gi & 63u));
  }
}

}  // namespace gv

extern "C" hipError_t gvk_verify_lat16(const gvk_lat* b, hipStream_t st) {
  const uint32_t blocks = (b->n + GV_LAT16_SIGS - 1) / GV_LAT16_SIGS;
  if (b->msg_blob) {
    hipError_t e = gvk_sha256(b->msg_blob, b->msg_off, b->msg_len, b->n, b->C, b->e_soa, st);
    if (e != hipSuccess) return e;
  }
  if (b->ev[0]) (void)hipEventRecord(b->ev[0], st);
  hipLaunchKernelGGL(gv::k_verify_lat16, dim3(blocks), dim3(128), 0, st, *b);
  return hipGetLastError();
}

extern "C" hipError_t gvk_verify_lat_sl(const gvk_lat* b, hipStream_t st) {
  // message path: the kernel's scalar wave hashes the sign bytes itself
  if (!b->out8) {
    hipError_t e = hipMemsetAsync(b->bits, 0, (size_t)((b->n + 63u) / 64u) * 8u, st);
    if (e != hipSuccess) return e;
  }
  if (b->ev[0]) (void)hipEventRecord(b->ev[0], st);
  if (b->gtab6) {                                      // the caller's choice (lat_rows_max)
    hipLaunchKernelGGL(gv::k_verify_lat_sl4, dim3(b->n), dim3(256), 0, st, *b);
    return hipGetLastError();
  }
  const uint32_t threads = b->n <= GV_LAT_SL_SPLIT ? 192u : 128u;
  hipLaunchKernelGGL(gv::k_verify_lat_sl, dim3(b->n), dim3(threads), 0, st, *b);
  return hipGetLastError();
}

extern "C" hipError_t gvk_verify_lat16_sl(const gvk_lat* b, hipStream_t st) {
  // message path: the kernel's scalar wave hashes the sign bytes itself
  if (!b->out8) {
    hipError_t e = hipMemsetAsync(b->bits, 0, (size_t)((b->n + 63u) / 64u) * 8u, st);
    if (e != hipSuccess) return e;
  }
  if (b->ev[0]) (void)hipEventRecord(b->ev[0], st);
  if (b->kn == 2 && b->gtab6) hipLaunchKernelGGL(gv::k_verify_lat16_kw, dim3(b->n), dim3(256), 0, st, *b);
  else if (b->kn && b->gtab6) hipLaunchKernelGGL(gv::k_verify_lat16_kn, dim3(b->n), dim3(256), 0, st, *b);
  else hipLaunchKernelGGL(gv::k_verify_lat16_sl, dim3(b->n), dim3(256), 0, st, *b);
  return hipGetLastError();
}

extern "C" hipError_t gvk_verify_lat(const gvk_lat* b, hipStream_t st) {
  const uint32_t blocks = (b->n + GV_LAT_SIGS - 1) / GV_LAT_SIGS;
  if (b->msg_blob) {
    hipError_t e = gvk_sha256(b->msg_blob, b->msg_off, b->msg_len, b->n, b->C, b->e_soa, st);
    if (e != hipSuccess) return e;
  }
  if (b->ev[0]) (void)hipEventRecord(b->ev[0], st);
  hipLaunchKernelGGL(gv::k_verify_lat, dim3(blocks), dim3(128), 0, st, b->gtab, b->pub33, b->sig64,
                     b->msg_blob ? nullptr : b->dig32, b->msg_blob ? (const uint32_t*)b->e_soa : nullptr,
                     b->C, b->n, (uint16_t*)b->bits, b->kslot, b->kqt, b->kzq, b->kok, b->kC, b->kcount);
  return hipGetLastError();
}

#if GV_LAT_TRACE
extern "C" int gv_debug_lat_trace(uint64_t* out, int blocks) {
  if (blocks > 256) blocks = 256;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(gv::g_lat_trace), (size_t)blocks * 8 * 8) == hipSuccess ? 0 : -3;
}
#endif
