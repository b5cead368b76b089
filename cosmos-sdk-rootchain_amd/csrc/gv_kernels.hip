// gv_kernels.hip -- the HIP/CDNA4 hot path of the batched secp256k1
// transaction-signature verifier (gfx950 / MI355X).
//
// Reference path being accelerated:
//   x/auth/ante/sigverify.go:210  pubKey.VerifyBytes(signBytes, sig)
//   -> tendermint v0.33.4 secp256k1_nocgo.go VerifyBytes
//   -> btcec.ParsePubKey / Signature.Verify -> go1.14 crypto/ecdsa.Verify
//
// Pipeline for a batch of C lanes (C = capacity rounded up to 256):
//   k_unpack      AoS bytes (pub33, sig64, dig32) -> SoA 32-bit limbs, via LDS
//   k_sha256      (message path) one StdSignBytes message per lane -> e limbs
//   k_scalar_inv  s^-1 mod n by Montgomery batch inversion (16 per lane + wave scan)
//   k_prep        pubkey decompression (sqrt), r/s/low-S range checks,
//                 u1 = e*w, u2 = r*w, GLV split of u1 and u2 (4 x 128-bit),
//                 signed (Booth) window digits, per-lane table of Q multiples
//                 (effective affine, shared Z)
//   k_ecmult      Strauss double-scalar multiplication: 5-bit windows for
//                 Q/lambda*Q from the lane's table, GV_GW-bit windows for G and
//                 lambda*G from two global tables (GV_GW=20: 32 MiB each); final
//                 x-coordinate check without inversion (X == r*Z^2 or
//                 (r+n)*Z^2); accept bitmap by ballot.
//
// SoA layout: limb i of item g lives at base[i*C + g] -> every per-limb access
// of a wave is one coalesced 256-byte transaction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "secp_field.cuh"
#include "secp_scalar.cuh"
#include "secp_group.cuh"
#include "secp_group29.cuh"
#include "secp_group29x.cuh"
#include "secp_sc29.cuh"
#include "secp_modinv.cuh"
#include "secp_sha256.cuh"
#include "gv_kernels.h"

namespace gv {

__constant__ const u32 kGx[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                                 0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
__constant__ const u32 kGy[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                                 0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
__constant__ const u32 kBeta[8] = {0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u,
                                   0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu};
// beta^2 mod p (the other cube root of unity: lambda^2 (x, y) = (beta^2 x, y))
__constant__ const u32 kBeta2[8] = {0x8E6AFA40u, 0x3EC693D6u, 0xED0A766Au, 0x630FB68Au,
                                    0x53CBCB16u, 0x919BB861u, 0x9A83F8EFu, 0x851695D4u};
__constant__ const u32 kP[8] = {0xFFFFFC2Fu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};

GV_DEV void load_fe(fe& r, const u32* base, u32 C, u32 g) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = base[(size_t)i * C + g];
}
GV_DEV void store_fe(u32* base, u32 C, u32 g, const fe& a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) base[(size_t)i * C + g] = a.v[i];
}
// 9 x 29 field elements cross memory as 8 x 32 words (value < 2^256,
// canonical when written here): the SoA rows and the 64-byte table entries
// keep one layout for both field layers.
GV_DEV void load_f29(fe29& r, const u32* base, u32 C, u32 g) {
  u32 w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = base[(size_t)i * C + g];
  f29_from_words(r, w);
}
GV_DEV void store_f29(u32* base, u32 C, u32 g, const fe29& a) {
  u32 w[8];
  f29_to_words(w, a);
#pragma unroll
  for (int i = 0; i < 8; ++i) base[(size_t)i * C + g] = w[i];
}
GV_DEV void f29_from_const(fe29& r, const u32* c) {
  u32 w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = c[i];
  f29_from_words(r, w);
}

GV_DEV void fe_from_const(fe& r, const u32* c) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = c[i];
}

// ---------------------------------------------------------------- k_gen_gtable
// gtab[e*16 + c]: e = 0..GV_GTAB_N-1 holds (e+1)*G affine, canonical; c = 0..7 x
// limbs, 8..15 y limbs; gtab[(GV_GTAB_N + e)*16 + c] holds (e+1)*lambda*G =
// (beta*x, y).  Run once per context.
// base: affine x || y (16 words) of the point whose multiples are tabulated,
// or null for G itself (the keyed ladder's tables of 2^35 G, 2^70 G, 2^100 G).
// GTN: entries per table (GV_GTAB_N; GV_K6_GTAB_N for the k6 tables).
// LAM false: the first table only (the full-scalar G tables).
template <u32 GTN = GV_GTAB_N, bool LAM = true>
__global__ void k_gen_gtable(u32* gtab, const u32* base) {
  const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= GTN) return;
  const u32 m = e + 1;
  fe gx, gy;
  if (base) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { gx.v[i] = base[i]; gy.v[i] = base[8 + i]; }
  } else {
    fe_from_const(gx, kGx);
    fe_from_const(gy, kGy);
  }
  gej acc;
  acc.x = gx; acc.y = gy; fe_set_u32(acc.z, 1);
  bool inf = false;
  int top = 31 - __builtin_clz(m);
  for (int b = top - 1; b >= 0; --b) {
    gej_double(acc, acc);
    if ((m >> b) & 1u) gej_add_ge(acc, inf, gx, gy);
  }
  fe zi, zi2, zi3, x, y;
  fe_inv(zi, acc.z);
  fe_sqr(zi2, zi);
  fe_mul(zi3, zi2, zi);
  fe_mul(x, acc.x, zi2);
  fe_mul(y, acc.y, zi3);
  fe_normalize(x);
  fe_normalize(y);
  u32* t0 = gtab + (size_t)e * 16;
#pragma unroll
  for (int i = 0; i < 8; ++i) { t0[i] = x.v[i]; t0[8 + i] = y.v[i]; }
  if (!LAM) return;
  fe beta, lx;
  fe_from_const(beta, kBeta);
  fe_mul(lx, x, beta);
  fe_normalize(lx);
  u32* t1 = gtab + ((size_t)GTN + e) * 16;
#pragma unroll
  for (int i = 0; i < 8; ++i) { t1[i] = lx.v[i]; t1[8 + i] = y.v[i]; }
}

// ------------------------------------------------------------------ k_unpack
// Stage nbytes of a row block into LDS with coalesced dword loads.
GV_DEV void stage_bytes(u32* lds, const uint8_t* src, u32 nbytes) {
  const u32 nw = nbytes >> 2;
  const u32* s32 = (const u32*)src;
  for (u32 i = threadIdx.x; i < nw; i += blockDim.x) lds[i] = s32[i];
  uint8_t* l8 = (uint8_t*)lds;
  for (u32 i = (nw << 2) + threadIdx.x; i < nbytes; i += blockDim.x) l8[i] = src[i];
}
GV_DEV u32 lds_be32(const uint8_t* p) {
  return ((u32)p[0] << 24) | ((u32)p[1] << 16) | ((u32)p[2] << 8) | (u32)p[3];
}

// pub33/sig64/dig32: device AoS inputs (dig32 may be null: message path;
// pub33 null: keyed batch; sig64 null: key load).
// Outputs (SoA, C lanes): x[8], pfx[1], r[8], s[8], e[8].  Lanes >= n get
// prefix 0 (rejected) and s = 1.
__global__ __launch_bounds__(256) void k_unpack(const uint8_t* pub33, const uint8_t* sig64,
                                                 const uint8_t* dig32, u32 n, u32 C,
                                                 u32* x, u32* pfx, u32* r, u32* s, u32* e) {
  __shared__ u32 lds[256 * 64 / 4];
  const u32 row0 = blockIdx.x * 256u;
  const u32 g = row0 + threadIdx.x;
  const u32 nv = (n > row0) ? min(256u, n - row0) : 0u;
  const bool live = threadIdx.x < nv;
  const uint8_t* l8 = (const uint8_t*)lds;

  if (pub33) {                    // null: keyed batch (cached keys) or signature-less key load
    stage_bytes(lds, pub33 + (size_t)row0 * 33u, nv * 33u);
    __syncthreads();
    const uint8_t* p = l8 + threadIdx.x * 33u;
    u32 pre = live ? p[0] : 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) x[(size_t)i * C + g] = live ? lds_be32(p + 1 + 4 * (7 - i)) : 0u;
    pfx[g] = pre;
  }
  if (sig64) {
    __syncthreads();
    stage_bytes(lds, sig64 + (size_t)row0 * 64u, nv * 64u);
    __syncthreads();
    const uint8_t* p = l8 + threadIdx.x * 64u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      r[(size_t)i * C + g] = live ? lds_be32(p + 4 * (7 - i)) : 0u;
      s[(size_t)i * C + g] = live ? lds_be32(p + 32 + 4 * (7 - i)) : (i == 0 ? 1u : 0u);
    }
  }
  if (dig32) {
    __syncthreads();
    stage_bytes(lds, dig32 + (size_t)row0 * 32u, nv * 32u);
    __syncthreads();
    const uint8_t* p = l8 + threadIdx.x * 32u;
#pragma unroll
    for (int i = 0; i < 8; ++i) e[(size_t)i * C + g] = live ? lds_be32(p + 4 * (7 - i)) : 0u;
  }
}

// ------------------------------------------------------------ in-batch keys
// A batch that repeats keys (a block with repeat signers; C2's 65,536 keys
// round-robin over 1M signatures) parses each distinct key once: the keys are
// grouped by an open-addressing hash table over the unpacked (prefix, x) rows,
// each distinct key gets an id, its tables are built once (k_keys_chain + k_keys_tables into a
// per-batch arena) and the items run the keyed pipeline (k_prep<true>,
// k_ecmult_k4) with the id as their slot.  ParsePubKey is a pure function of
// the 33 bytes, so the verdicts are the per-item ones (SURVEY.md §8f-2 within
// one batch).
GV_DEV u32 key_hash(const u32 w[8], u32 pre) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ pre;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h ^= w[i];
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 29;
  }
  return (u32)(h ^ (h >> 32));
}
GV_DEV bool key_equal(const u32* x, const u32* pfx, u32 C, u32 a, u32 b) {
  bool eq = pfx[a] == pfx[b];
#pragma unroll
  for (int i = 0; i < 8; ++i) eq &= x[(size_t)i * C + a] == x[(size_t)i * C + b];
  return eq;
}
// rep[g] = the first-inserted item with g's key (table: tmask + 1 slots of
// 0xFFFFFFFF, at least twice the items).  A key ParsePubKey rejects on its
// bytes alone -- prefix not 02/03, x >= p -- gets no id and no tables:
// rep[g] = 0xFFFFFFFF, and k_dedupe_map gives its items an out-of-range slot,
// which the keyed pipeline answers false (the adversarial mix's malformed
// keys are distinct per item: each would otherwise cost a table build).
__global__ __launch_bounds__(256) void k_dedupe(u32 n, u32 C, const u32* x, const u32* pfx, u32* table, u32 tmask,
                                                 u32* rep) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  u32 w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = x[(size_t)i * C + g];
  {
    u32 br = 0, d;
#pragma unroll
    for (int i = 0; i < 8; ++i) d = __builtin_subc(w[i], kP[i], br, &br);
    (void)d;
    if ((pfx[g] & 0xFEu) != 0x02u || br == 0u) { rep[g] = 0xFFFFFFFFu; return; }   // x >= p: no borrow
  }
  for (u32 sl = key_hash(w, pfx[g]) & tmask;; sl = (sl + 1) & tmask) {
    const u32 cur = atomicCAS(&table[sl], 0xFFFFFFFFu, g);
    if (cur == 0xFFFFFFFFu) { rep[g] = g; return; }
    if (key_equal(x, pfx, C, cur, g)) { rep[g] = cur; return; }
  }
}
// Each representative takes the next key id; its (prefix, x) goes to key row
// id (stride CU) when id < capU (a batch with more distinct keys takes the
// pub33 pipeline and never reads these rows).
__global__ __launch_bounds__(256) void k_dedupe_assign(u32 n, u32 C, const u32* x, const u32* pfx, const u32* rep,
                                                        u32* uid, u32* count, u32 capU, u32 CU, u32* kx, u32* kpfx) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  const bool first = g < n && rep[g] == g;
  // one atomic per wave: the wave's representatives take consecutive ids
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
#pragma unroll
    for (int i = 0; i < 8; ++i) kx[(size_t)i * CU + u] = x[(size_t)i * C + g];
    kpfx[u] = pfx[g];
  }
}
__global__ __launch_bounds__(256) void k_dedupe_map(u32 n, const u32* rep, const u32* uid, u32* kslot) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n) kslot[g] = rep[g] == 0xFFFFFFFFu ? 0xFFFFFFFFu : uid[rep[g]];
}

// ------------------------------------------------------------------ k_sha256
// perm (nullable): lane g hashes item perm[g] (key-ordered lanes, gv_sort.hip)
__global__ __launch_bounds__(256) void k_sha256(const uint8_t* blob, const uint64_t* off,
                                                 const u32* len, u32 n, u32 C, u32* e, const u32* perm) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= C) return;
  u32 h[8];
  if (g < n) {
    const u32 i = perm ? perm[g] : g;
    sha256_msg(h, blob + off[i], len[i]);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = 0;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) e[(size_t)i * C + g] = h[7 - i];
}

// ------------------------------------------------------------ ladder helpers
// One lane's Q table: m*Q for m = 1..GV_QTAB_N in the isomorphic-curve affine
// representation with a shared Z (returned in zq).  qt layout: the first
// C*16*16 words hold the entries lane-major (AoS): lane g, entry m at
// qt[(g*16 + m-1)*16 ..], x then y, 64 contiguous bytes, so k_ecmult's
// per-lane gather of an entry is four 16-byte loads instead of sixteen 4-byte
// loads spread over sixteen lines.  The Z-ratio scratch follows as SoA rows:
// qr[(i*8 + c) * C + g].
//
// Built with co-Z arithmetic (Meloni's ZADDU): a co-Z doubling gives 2Q and
// Q' (Q on the same Z); then each step adds the co-Z pair (Q', mQ) into
// (m+1)Q and re-expresses Q' on the new Z, for 4M + 2S per step (the new Z,
// Z*(X1-X2), is never formed: only the ratio X1-X2 is stored).  No exceptional
// case: X(Q') == X(mQ) would need mQ == +-Q, i.e. n | m -+ 1, for 2 <= m <= 15.
// Every entry is then scaled to the last entry's Z by back-propagating the
// ratios, and zq = 2y * prod(ratios) is that Z.
GV_DEV void store_qent(u32* qt, u32 g, int j, const fe& x, const fe& y) {
  uint4* p = (uint4*)(qt + ((size_t)g * GV_QTAB_N + j) * 16);
  p[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
  p[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
  p[2] = make_uint4(y.v[0], y.v[1], y.v[2], y.v[3]);
  p[3] = make_uint4(y.v[4], y.v[5], y.v[6], y.v[7]);
}
GV_DEV void load_qent(fe& x, fe& y, const u32* qt, u32 g, u32 j) {
  const uint4* p = (const uint4*)(qt + ((size_t)g * GV_QTAB_N + j) * 16);
  uint4 a = p[0], b = p[1], c = p[2], d = p[3];
  x.v[0] = a.x; x.v[1] = a.y; x.v[2] = a.z; x.v[3] = a.w;
  x.v[4] = b.x; x.v[5] = b.y; x.v[6] = b.z; x.v[7] = b.w;
  y.v[0] = c.x; y.v[1] = c.y; y.v[2] = c.z; y.v[3] = c.w;
  y.v[4] = d.x; y.v[5] = d.y; y.v[6] = d.z; y.v[7] = d.w;
}

// Q-table entries (built and read on the 9 x 29 layer) are stored as raw
// limbs: x[9], y[9], 2 pad words = 80 bytes, five 16-byte accesses per lane;
// no word conversion on either side.  G-table entries stay 8 x 32 words.
// NT: entries per table row (GV_QTAB_N; GV_K6_NT for the k6 group tables).
// EW: words per entry (GV_QENT_WORDS; the wide arena may pad to a cache line).
// EW == 16: the entry as canonical words x[8] y[8] (64 B, one half line),
// converted on both sides.
template <int NT = GV_QTAB_N, int EW = GV_QENT_WORDS>
GV_DEV void store_qent29(u32* qt, u32 g, int j, const fe29& x, const fe29& y) {
  uint4* p = (uint4*)(qt + ((size_t)g * NT + j) * EW);
  if constexpr (EW == 16) {
    u32 xw[8], yw[8];
    f29_to_words(xw, x);
    f29_to_words(yw, y);
    p[0] = make_uint4(xw[0], xw[1], xw[2], xw[3]);
    p[1] = make_uint4(xw[4], xw[5], xw[6], xw[7]);
    p[2] = make_uint4(yw[0], yw[1], yw[2], yw[3]);
    p[3] = make_uint4(yw[4], yw[5], yw[6], yw[7]);
    return;
  }
  p[0] = make_uint4(x.n[0], x.n[1], x.n[2], x.n[3]);
  p[1] = make_uint4(x.n[4], x.n[5], x.n[6], x.n[7]);
  p[2] = make_uint4(x.n[8], y.n[0], y.n[1], y.n[2]);
  p[3] = make_uint4(y.n[3], y.n[4], y.n[5], y.n[6]);
  p[4] = make_uint4(y.n[7], y.n[8], 0u, 0u);
}
template <int NT = GV_QTAB_N, int EW = GV_QENT_WORDS>
GV_DEV void load_qent29(fe29& x, fe29& y, const u32* qt, u32 g, u32 j) {
  const uint4* p = (const uint4*)(qt + ((size_t)g * NT + j) * EW);
  if constexpr (EW == 16) {
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    const u32 xw[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const u32 yw[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
    f29_from_words(x, xw);
    f29_from_words(y, yw);
    return;
  }
  const uint4 a = p[0], b = p[1], c = p[2], d = p[3], e = p[4];
  x.n[0] = a.x; x.n[1] = a.y; x.n[2] = a.z; x.n[3] = a.w;
  x.n[4] = b.x; x.n[5] = b.y; x.n[6] = b.z; x.n[7] = b.w;
  x.n[8] = c.x; y.n[0] = c.y; y.n[1] = c.z; y.n[2] = c.w;
  y.n[3] = d.x; y.n[4] = d.y; y.n[5] = d.z; y.n[6] = d.w;
  y.n[7] = e.x; y.n[8] = e.y;
}
GV_DEV void load_gent29(fe29& x29, fe29& y29, const u32* gt, u32 j) {
  fe x, y;
  load_qent(x, y, gt, 0, j);
  f29_from_words(x29, x.v);
  f29_from_words(y29, y.v);
}
// Z-ratio scratch: 9 raw-limb SoA rows per ratio after the entries.
GV_DEV void store_ratio29(u32* qr, u32 C, u32 g, int k, const fe29& a) {
#pragma unroll
  for (int i = 0; i < 9; ++i) qr[((size_t)k * 9 + i) * C + g] = a.n[i];
}
GV_DEV void load_ratio29(fe29& a, const u32* qr, u32 C, u32 g, int k) {
#pragma unroll
  for (int i = 0; i < 9; ++i) a.n[i] = qr[((size_t)k * 9 + i) * C + g];
}

// Magnitudes (9 x 29 layer) annotated per step; every stored value is
// canonical words.
// qt: entries of table row qi (lane-major AoS); qr: Z-ratio scratch rows of
// stride C, column g.
GV_DEV void build_q_table(u32* qt, u32 qi, u32* qr, u32 C, u32 g, const fe& qx8, const fe& qy8, fe& zq8) {
  fe29 qx, qy, X1, Y1, X2, Y2, t, u;
  f29_from_words(qx, qx8.v);
  f29_from_words(qy, qy8.v);
  {
    // co-Z doubling of the affine Q: Z1 = 2y, 2Q = (M^2 - 2S, M(S - X) - 8y^4),
    // Q' = (S, 8y^4) with S = 4xy^2, M = 3x^2.
    fe29 B, E, L, M;
    f29_sqr(B, qx);                                   // 1
    f29_sqr(E, qy);                                   // 1
    f29_sqr(L, E);                                    // y^4: 1
    f29_add(t, qx, E);                                // 2
    f29_sqr(t, t);                                    // 1
    f29_sub<1>(t, t, B);                              // 3
    f29_sub_norm<1>(t, t, L);                         // (x + y^2)^2 - x^2 - y^4 = 2xy^2: 1
    f29_shl_norm<1>(X1, t);                           // S = 4xy^2: 1
    f29_mul3_norm(M, B);                              // 1
    f29_sqr(t, M);                                    // 1
    f29_add(u, X1, X1);                               // 2
    f29_sub_norm<2>(X2, t, u);                        // M^2 - 2S: 1
    f29_shl_norm<3>(Y1, L);                           // 8y^4: 1
    f29_sub<1>(t, X1, X2);                            // 3
    f29_mul(t, M, t);                                 // 1
    f29_sub_norm<1>(Y2, t, Y1);                       // 1
  }
  store_qent29(qt, qi, 0, X1, Y1);                     // 1*Q on Z1
  store_qent29(qt, qi, 1, X2, Y2);                     // 2*Q on Z1
  for (int m = 2; m < GV_QTAB_N; ++m) {               // (Q', mQ) -> ((m+1)Q, Q'')
    fe29 h, rr, c, w1, w2, d, a1;
    f29_sub_norm<1>(h, X1, X2);                       // 1
    store_ratio29(qr, C, g, m - 2, h);                // Z_m / Z_{m-1}
    f29_sub_norm<1>(rr, Y1, Y2);                      // 1
    f29_sqr(c, h);
    f29_mul(w1, X1, c);
    f29_mul(w2, X2, c);
    f29_sqr(d, rr);
    f29_sub<1>(t, w1, w2);                            // 3
    f29_mul(a1, Y1, t);                               // 1
    f29_add(u, w1, w2);                               // 2
    f29_sub_norm<2>(X2, d, u);                        // X3 = D - W1 - W2: 1
    f29_sub<1>(t, w1, X2);                            // 3
    f29_mul(t, rr, t);                                // 1
    f29_sub_norm<1>(Y2, t, a1);                       // Y3 = (Y1-Y2)(W1-X3) - A1: 1
    X1 = w1;                                          // Q' on the new Z
    Y1 = a1;
    store_qent29(qt, qi, m, X2, Y2);                   // (m+1)*Q
  }
  // entry m (index m-1) lives on Z_{m-1} (m >= 2; entry 1 on Z_1); the last
  // entry on Z_15.  acc = Z_15 / Z(entry m) accumulates the stored ratios.
  fe29 acc;
  for (int m = GV_QTAB_N - 1; m >= 1; --m) {
    if (m >= 2) {
      fe29 ratio;
      load_ratio29(ratio, qr, C, g, m - 2);
      if (m == GV_QTAB_N - 1) acc = ratio;
      else f29_mul(acc, acc, ratio);
    }
    fe29 x, y, a2, a3;
    f29_sqr(a2, acc);
    f29_mul(a3, a2, acc);
    load_qent29(x, y, qt, qi, m - 1);
    f29_mul(x, x, a2);
    f29_mul(y, y, a3);
    store_qent29(qt, qi, m - 1, x, y);
  }
  f29_add(t, qy, qy);                                 // 2
  f29_mul(t, t, acc);                                 // Z_15 = 2y * prod(ratios)
  f29_to_words(zq8.v, t);
}

// GV_FRONT_VGPR: VGPR cap of the front kernels (k_keys_chain, k_keys_tables,
// k_scalar_inv), so that a front wave fits beside three ladder waves
// (k_ecmult_k4 / k6: 134 VGPRs) and the next call's front runs under the
// current ladder instead of after it (0: compiler's choice).
#ifndef GV_FRONT_VGPR
#define GV_FRONT_VGPR 0
#endif
#if GV_FRONT_VGPR
#define GV_FRONT_ATTR __attribute__((amdgpu_waves_per_eu(512 / GV_FRONT_VGPR)))
#else
#define GV_FRONT_ATTR
#endif
// GV_SINV_VGPR: the same cap for k_scalar_inv alone (96: it then fits beside
// three ladder waves of 136 allocated VGPRs; A/B)
#ifndef GV_SINV_VGPR
#define GV_SINV_VGPR 0
#endif
#if GV_SINV_VGPR
#define GV_SINV_ATTR __attribute__((amdgpu_waves_per_eu(512 / GV_SINV_VGPR)))
#else
#define GV_SINV_ATTR GV_FRONT_ATTR
#endif
// ------------------------------------------------------------- k_scalar_inv
// w = s^-1 mod n for every lane, Montgomery form (radix 2^29, R = 2^261,
// secp_sc29.cuh), by Montgomery's trick: each lane folds GV_INV_M signatures
// (element (wave*M + j)*64 + lane, so each step j is a coalesced wave access),
// the lane totals are combined across the wavefront by prefix/suffix scans,
// and ONE Fermat inversion serves the wave's 64*M signatures -- ~3 Montgomery
// products per signature + ~330/M amortised, instead of ~330 (a per-lane
// inversion costs the same SIMT time whether one lane or all 64 run it).  s
// outside [1, n) is replaced by 1 (those lanes are rejected in k_prep).
// w and the prefix products use 9 scratch rows each (limb i of lane e at
// row[i*C + e]); the caller gives the row bases.
GV_DEV void load_sc(u32 a[8], const u32* base, u32 C, u32 g) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = base[(size_t)i * C + g];
}
GV_DEV void load_sc29(sc29& a, const u32* base, u32 C, u32 g) {
#pragma unroll
  for (int i = 0; i < 9; ++i) a.n[i] = base[(size_t)i * C + g];
}
GV_DEV void store_sc29(u32* base, u32 C, u32 g, const sc29& a) {
#pragma unroll
  for (int i = 0; i < 9; ++i) base[(size_t)i * C + g] = a.n[i];
}
GV_DEV void sc29_mont_one(sc29& r) {          // R mod n = 2^261 mod n
  const u32 t[9] = {0x1937D7E0u, 0x0DA1732Fu, 0x1AFE2201u, 0x08C6542Du, 0x00028AA2u, 0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < 9; ++i) r.n[i] = t[i];
}
GV_DEV sc29 sc29_shfl(const sc29& a, int mode, int d) {
  sc29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i)
    r.n[i] = mode == 0 ? shfl_up_u32(a.n[i], d) : mode == 1 ? shfl_down_u32(a.n[i], d) : shfl_idx_u32(a.n[i], d);
  return r;
}

// GV_SINV_DIVSTEPS (default 1): the shared inversion by var-time divsteps
// instead of the Fermat chain s^(n-2) (0: A/B).
#ifndef GV_SINV_DIVSTEPS
#define GV_SINV_DIVSTEPS 1
#endif
// Batch inversion across the wavefront: every lane holds a nonzero x
// (Montgomery form); returns x^-1 (Montgomery form).  All 64 lanes active.
// Prefix/suffix products by Hillis-Steele scans (6 steps each) + one Fermat
// inversion shared by the wave.
GV_DEV void sc29_batch_inv_wave(sc29& inv, const sc29& x) {
  const u32 lane = lane_id();
  sc29 pre = x, suf = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    sc29 t = sc29_shfl(pre, 0, d), m;
    sc29_mul(m, pre, t);
#pragma unroll
    for (int i = 0; i < 9; ++i) pre.n[i] = (lane >= (u32)d) ? m.n[i] : pre.n[i];
    t = sc29_shfl(suf, 1, d);
    sc29_mul(m, suf, t);
#pragma unroll
    for (int i = 0; i < 9; ++i) suf.n[i] = (lane + (u32)d < 64u) ? m.n[i] : suf.n[i];
  }
  sc29 tot = sc29_shfl(pre, 2, 63), tinv, one;
#if GV_SINV_DIVSTEPS
  {
    // every lane inverts the same total, so the variable-time divsteps
    // (secp_modinv.cuh, ~1/10 of the Fermat chain's instructions) never
    // diverge: Montgomery -> plain, x^-1, plain -> Montgomery
    sc29 p1, xp;
#pragma unroll
    for (int i = 0; i < 9; ++i) p1.n[i] = i == 0 ? 1u : 0u;
    sc29_mul(xp, tot, p1);                     // tot * 1 / R = x
    u32 xw[8], iw[8];
    sc29_to_words(xw, xp);
    s30_modinv_var(iw, xw, []() {});
    sc29 ip;
    sc29_from_words(ip, iw);
    sc29_to_mont(tinv, ip);
  }
#else
  sc29_inv(tinv, tot);
#endif
  sc29_mont_one(one);
  sc29 pe = sc29_shfl(pre, 0, 1), se = sc29_shfl(suf, 1, 1), m;
  if (lane == 0) pe = one;
  if (lane == 63) se = one;
  sc29_mul(m, pe, se);
  sc29_mul(inv, m, tinv);
}

// M: signatures per lane (GV_INV_M for large batches; fewer for a batch whose
// s^-1 is on a latency path, gvk_inv_m).
__global__ __launch_bounds__(256) GV_SINV_ATTR void k_scalar_inv(u32 C, const u32* in_s, u32* w, u32* pre, u32 M) {
  const u32 lane = threadIdx.x & 63u;
  const u32 wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  sc29 acc;
  sc29_mont_one(acc);
  for (u32 j = 0; j < M; ++j) {
    const u32 e = (wave * M + j) * 64u + lane;
    if (e >= C) break;                       // wave-uniform (C % 64 == 0)
    u32 s[8];
    load_sc(s, in_s, C, e);
    const bool ok = !u256_is_zero(s) && !u256_geq(s, kN);
    if (!ok) {
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] = (i == 0) ? 1u : 0u;
    }
    sc29 s29, sm;
    sc29_from_words(s29, s);
    sc29_to_mont(sm, s29);
    store_sc29(pre, C, e, acc);              // exclusive prefix within the lane
    store_sc29(w, C, e, sm);
    sc29_mul(acc, acc, sm);
  }
  sc29 inv_lane;
  sc29_batch_inv_wave(inv_lane, acc);        // (lane total)^-1, one Fermat chain per wave
  for (int j = (int)M - 1; j >= 0; --j) {
    const u32 e = (wave * M + (u32)j) * 64u + lane;
    if (e >= C) continue;
    sc29 p, sm, inv;
    load_sc29(p, pre, C, e);
    load_sc29(sm, w, C, e);
    sc29_mul(inv, inv_lane, p);              // s_j^-1 = (s_0..s_j)^-1 * (s_0..s_{j-1})
    sc29_mul(inv_lane, inv_lane, sm);        // drop s_j from the running inverse
    store_sc29(w, C, e, inv);
  }
}

// -------------------------------------------------------------------- k_prep
// btcec.ParsePubKey for a compressed key (prefix 02/03, x < p, decompressPoint:
// y = sqrt(x^3 + 7) with the prefix's parity; IsOnCurve and y < p then hold by
// construction).  Returns false for a rejected key (x, y then undefined).
GV_DEV bool parse_pubkey(u32 pre, const fe& x, fe& y) {
  bool ok = (pre & 0xFEu) == 0x02u;
  {                                         // x < p  (btcec: "pubkey X parameter is >= to P")
    u32 br = 0, d;
#pragma unroll
    for (int i = 0; i < 8; ++i) d = __builtin_subc(x.v[i], kP[i], br, &br);
    (void)d;
    ok &= (br != 0);
  }
  {
    fe29 x29, c, y29, y2, seven;
    f29_from_words(x29, x.v);
    f29x_sqr(c, x29);
    f29x_mul(c, c, x29);
    f29_set_u32(seven, 7);
    f29_add(c, c, seven);                   // c = x^3 + 7 (magnitude 2)
    f29x_sqrt_candidate(y29, c);            // y = c^((p+1)/4)
    f29x_sqr(y2, y29);
    ok &= f29_equal(y2, c);                 // "invalid square root"
    f29_to_words(y.v, y29);                 // canonical
  }
  if ((y.v[0] & 1u) != (pre & 1u)) fe_neg(y, y);   // choose parity (y != 0 always)
  fe_normalize(y);
  return ok;
}

// flags bits: 1 = passes every check before the curve arithmetic,
//             2 = r < p - n (so R.x == r + n is also an accept)
// KEYED = false: the lane's pubkey (in_x, in_pfx) is parsed here and its Q
// table built into qt row g (zq_out column g).
// KEYED = true: the item's key is slot kslot[g] of the key arena (gv_keys_load:
// parsed once, table resident); an out-of-range slot or a rejected key makes
// the item false.  qidx[g] receives the (clamped) slot for k_ecmult.
// GV_PREP_WAVES: minimum waves per SIMD for k_prep (0 = compiler's choice; A/B)
#ifndef GV_PREP_WAVES
#define GV_PREP_WAVES 0
#endif
#if GV_PREP_WAVES
#define GV_PREP_ATTR __attribute__((amdgpu_waves_per_eu(GV_PREP_WAVES)))
#else
#define GV_PREP_ATTR
#endif
// K6 (keyed only): the digits of the k6 ladder (GV_K6_QW-bit Q windows,
// GV_K6_GW-bit G windows) instead of GV_QW / GV_GW.
// GF (keyed k4 only): G digits of the unsplit u1 (GV_GF_WIN signed
// GV_GF_W-bit windows, one int32 row each: digits[(GV_QWIN + j)*C + g]).
// KW (with K6, GF): GV_KW_QW-bit Q windows (the resident arena's wide-window
// tables), G as K6.
// KG (with K6, GF): GV_QW-bit Q windows (the grouped route's many-group
// tables, option "kg"), G as K6.
template <bool KEYED, bool K6 = false, bool GF = false, bool KW = false, bool KG = false>
__global__ __launch_bounds__(256) GV_PREP_ATTR void k_prep(u32 C, u32 n, const u32* in_x, const u32* in_pfx,
                                               const u32* in_r, const u32* in_s, const u32* in_e,
                                               const u32* in_w, u32* digits, u32* qt, u32* zq_out,
                                               u32* flags, const u32* kslot, const u32* kok, u32 kcount,
                                               u32* qidx) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;   // C % 256 == 0: all lanes live
  bool ok = true;
  fe x, y;
  if (KEYED) {
    u32 sl = g < n ? kslot[g] : 0xFFFFFFFFu;
    const bool in_range = sl < kcount;
    if (!in_range) sl = 0;                  // the arena always holds slot 0's memory
    ok = in_range && kok[sl] != 0u;
    qidx[g] = sl;
  } else {
    load_fe(x, in_x, C, g);
    ok = parse_pubkey(in_pfx[g], x, y);
  }

  // ---- tendermint low-S + crypto/ecdsa range checks
  u32 r[8], s[8], e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r[i] = in_r[(size_t)i * C + g];
    s[i] = in_s[(size_t)i * C + g];
    e[i] = in_e[(size_t)i * C + g];
  }
  ok &= !u256_is_zero(r);
  ok &= !u256_geq(r, kN);
  ok &= !u256_is_zero(s);
  ok &= u256_geq(kHalfN, s);                // s <= N/2  (tendermint rejects s > halfN)
  // r < p - n ?
  const bool r_small = !u256_geq(r, kPminusN);
  sc_reduce_once(e);                        // e mod n (hashToInt keeps all 256 bits)

  // invalid lanes: harmless stand-ins so the whole wave stays on one path
  if (!ok) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { s[i] = (i == 0) ? 1u : 0u; e[i] = 0u; r[i] = 0u; }
    if (!KEYED) {
      fe_from_const(x, kGx);
      fe_from_const(y, kGy);
    }
  }

  // ---- w = s^-1 mod n (Montgomery form, from k_scalar_inv)
  u32 u1[8], u2[8];
  {
    sc29 w29, e29, r29, t;
    load_sc29(w29, in_w, C, g);
    sc29_from_words(e29, e);
    sc29_from_words(r29, r);
    sc29_mul(t, e29, w29);                  // e*w  (plain form)
    sc29_to_words(u1, t);
    sc29_mul(t, r29, w29);                  // r*w
    sc29_to_words(u2, t);
  }

  // ---- GLV split
  u32 k1g[4] = {}, k2g[4] = {}, k1q[4], k2q[4], n1g = 0, n2g = 0, n1q, n2q;
  if (!GF) glv_split(k1g, n1g, k2g, n2g, u1);
  glv_split(k1q, n1q, k2q, n2q, u2);
  if (!ok) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { k1g[i] = k2g[i] = k1q[i] = k2q[i] = 0u; }
#pragma unroll
    for (int i = 0; i < 8; ++i) u1[i] = 0u;
  }

  // ---- signed fixed-window (Booth) recoding, scalar signs folded in.
  // Q digits (5-bit windows, [-16, 16]): digits[win*C + g] = dQ1 | dQ2 << 16
  // (int16 halves), win = 0..GV_QWIN-1.  G digits (GV_GW-bit windows,
  // [-2^(GV_GW-1), 2^(GV_GW-1)]) as int32: digits[(GV_QWIN + 2j)*C + g] = dG1,
  // digits[(GV_QWIN + 2j + 1)*C + g] = dG2, j = 0..GV_GWIN-1.
  static_assert(GF || !K6, "the k6 ladder takes G on the unsplit scalar");
  static_assert(!KW || K6, "wide-window digits: the k6 ladder's G windows");
  static_assert(!KG || (K6 && !KW), "kg digits: 5-bit Q windows, the k6 ladder's G windows");
  constexpr int QW = KW ? GV_KW_QW : KG ? GV_QW : K6 ? GV_K6_QW : GV_QW;
  constexpr int QWIN = KW ? GV_KW_QWIN : KG ? GV_QWIN : K6 ? GV_K6_QWIN : GV_QWIN;
  constexpr int GW = GV_GW, GWIN = GV_GWIN;
  constexpr int GFW = K6 ? GV_K6_GW : GV_GF_W, GFWIN = K6 ? GV_K6_GWIN : GV_GF_WIN;
#pragma unroll
  for (int win = 0; win < QWIN; ++win) {
    int d0 = booth_digit<QW>(k1q, win), d1 = booth_digit<QW>(k2q, win);
    if (n1q) d0 = -d0;
    if (n2q) d1 = -d1;
    digits[(size_t)win * C + g] = ((u32)d0 & 0xFFFFu) | ((u32)d1 << 16);
  }
  if (GF) {
#pragma unroll
    for (int j = 0; j < GFWIN; ++j) digits[(size_t)(QWIN + j) * C + g] = (u32)booth_digit8<GFW>(u1, j);
  } else {
#pragma unroll
    for (int j = 0; j < GWIN; ++j) {
      int d2 = booth_digit<GW>(k1g, j), d3 = booth_digit<GW>(k2g, j);
      if (n1g) d2 = -d2;
      if (n2g) d3 = -d3;
      digits[(size_t)(QWIN + 2 * j) * C + g] = (u32)d2;
      digits[(size_t)(QWIN + 2 * j + 1) * C + g] = (u32)d3;
    }
  }
  flags[g] = (ok ? 1u : 0u) | (r_small ? 2u : 0u);

  // ---- per-lane table of Q multiples (shared Z, isomorphic-curve affine)
  if (!KEYED) {
    fe zq;
    build_q_table(qt, g, qt + (size_t)C * GV_QTAB_N * GV_QENT_WORDS, C, g, x, y, zq);
    store_fe(zq_out, C, g, zq);
  }
}

// ------------------------------------------------------------ key tables
#ifndef GV_KEYS_PREFETCH
#define GV_KEYS_PREFETCH 1
#endif
// Key arena (gv_keys_load): lane g parses key g of the load batch once and
// writes its Q table to arena row base + g, the table's Z to kzq (8 rows of
// stride kC) and the ParsePubKey verdict to kok.  A rejected key gets G's
// table (never used: every item against it is false).  qr: Z-ratio scratch
// rows of stride C.
// Window-group start bits of the keyed latency schedule (GV_LGRP groups).
__constant__ const int kLGrpBit[GV_LGRP] = {0, 35, 70, 100};

// Group layout of the keyed throughput ladders (gv_kernels.h): QWIN signed
// QW-bit windows per 128-bit GLV half split into NG groups -- the first R of
// P = ceil(QWIN / NG) windows, the rest of P - 1 -- group k starting at window
// w0(k), i.e. its table is that of 2^(QW w0(k)) Q; the ladder runs P
// positions.  <5, 4>: k_ecmult_k4 (groups at bits 0, 35, 70, 100); <6, 4>:
// the grouped route's k6 (0, 36, 72, 102); <6, GV_KN_ARENA_NG> and
// <GV_KW_QW, GV_KW_NG1 / GV_KW_NG2>: the resident arena's table sets.
template <int QW, int NG>
struct KLayout {
  static constexpr int QWIN = QW == GV_QW ? GV_QWIN : QW == GV_KW_QW ? GV_KW_QWIN : GV_K6_QWIN;
  static constexpr int NT = 1 << (QW - 1);                  // table entries per group
  static constexpr int EW = QW == GV_KW_QW ? GV_KW_ENT_WORDS : GV_QENT_WORDS;   // words per entry
  static constexpr int P = (QWIN + NG - 1) / NG;            // ladder positions
  static constexpr int R = QWIN - (P - 1) * NG;             // groups with P windows
  static constexpr int nw(int k) { return k < R ? P : P - 1; }
  static constexpr int w0(int k) { return k * P - (k > R ? k - R : 0); }
  static constexpr int bit(int k) { return QW * w0(k); }
};
static_assert(KLayout<5, 4>::bit(1) == 35 && KLayout<5, 4>::bit(2) == 70 && KLayout<5, 4>::bit(3) == 100 &&
              KLayout<5, 4>::P == 7, "k4 groups");
static_assert(KLayout<6, 4>::bit(1) == 36 && KLayout<6, 4>::bit(2) == 72 && KLayout<6, 4>::bit(3) == 102 &&
              KLayout<6, 4>::P == 6, "k6 groups");
static_assert(KLayout<6, GV_KN_ARENA_NG>::w0(GV_KN_ARENA_NG - 1) + KLayout<6, GV_KN_ARENA_NG>::nw(GV_KN_ARENA_NG - 1) ==
              GV_K6_QWIN, "arena groups cover the windows");
static_assert(KLayout<GV_KW_QW, GV_KW_NG2>::w0(GV_KW_NG2 - 1) + KLayout<GV_KW_QW, GV_KW_NG2>::nw(GV_KW_NG2 - 1) ==
                      GV_KW_QWIN && KLayout<GV_KW_QW, GV_KW_NG2>::P == 2 && KLayout<GV_KW_QW, GV_KW_NG1>::P == 1,
              "wide arena groups cover the windows");

// Affine x, y (8 x 32 words) of a finite Jacobian point.
GV_DEV void gej29_to_affine_words(fe& x8, fe& y8, const gej29& p) {
  fe29 zi, z2, z3, x, y;
  f29_inv(zi, p.z);
  f29_sqr(z2, zi);
  f29_mul(z3, z2, zi);
  f29_mul(x, p.x, z2);
  f29_mul(y, p.y, z3);
  f29_to_words(x8.v, x);
  f29_to_words(y8.v, y);
}

// The keyed ladders' tables are built in three launches so that the long
// serial part runs one lane per key and the rest one lane per (key, group):
//
// k_keys_chain: ParsePubKey and the doublings to each group's base 2^bit(k) Q
// (100 for k4), on two waves per key set so the square root is off the
// doubling chain (round 6).  With c = x^3 + 7 the point Q' = (c x, c^2) lies
// on E': Y^2 = X^3 + 7 c^3, the image of Q = (x, y) under (x, y) -> (u^2 x,
// u^3 y) with u = y (u^2 = c): a = 0 doubling and addition formulas never read
// the curve constant, so the chain and the tables run on Q' as soon as c is
// known, and a Jacobian (X, Y, Z) of E' is the point (X, Y, u Z) of E.
// Blocks of 256 keys in 512 threads: waves 0-3 (the root role) run
// ParsePubKey's checks and square root -- the verdict to kok, u (the root with
// the prefix's parity) to the key's Z row kzq, which k_keys_fwd /
// k_keys_tables fold into every group's table Z; waves 4-7 (the chain role)
// park Q' and its doublings.  A block's wave w runs on SIMD w % 4, so every
// SIMD holds one root wave beside one chain wave: the chain's dependent
// products interleave with the root's instead of waiting on themselves.  For
// a key ParsePubKey rejects c may be a non-square (Q' on the twist): its tables
// are computed all the same and never used -- every item against it is false.
// Each group's base point is parked, as canonical words x[8] y[8], in entry 0
// of its own table row (group 0 in kqt, groups 1.. in kqt2 rows slot * (NG -
// 1) + k - 1); the Jacobian Z of groups 1.. in their Z rows (kzq2, (NG - 1) x
// 8 rows of stride kC), group 0 is affine (on E').
// GV_CHAIN_SPLIT 0 (the default): one lane per key runs ParsePubKey, then
// the doublings on E itself (u = 1 in kzq), as in rounds 3-5.  1: the root
// and chain roles above -- the serialized key stage is ~10 % shorter, but the
// pipelined C2 step loses 4-5 % (216 vs 226M/s alternated on one box,
// profiles/r06/ab/ab3): the 512-thread blocks wait for two free wave slots on
// every SIMD of a CU, which the previous call's ladder holds.
#ifndef GV_CHAIN_SPLIT
#define GV_CHAIN_SPLIT 0
#endif
template <int QW, int NG>
__global__ __launch_bounds__(512) GV_FRONT_ATTR void k_keys_chain(u32 n, u32 C, const u32* in_x, const u32* in_pfx, u32 base,
                                                     u32* kqt, u32 kC, u32* kok, u32* kqt2, u32* kzq2, u32* kzq) {
  using L = KLayout<QW, NG>;
#if GV_CHAIN_SPLIT
  const bool root = threadIdx.x < 256u;                 // wave-uniform role
  const u32 g = blockIdx.x * 256u + (threadIdx.x & 255u);
#else
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
#endif
  if (g >= n) return;                       // no cross-lane work
#if !GV_CHAIN_SPLIT
  {
    fe x, y;
    load_fe(x, in_x, C, g);
    const bool ok = parse_pubkey(in_pfx[g], x, y);
    if (!ok) {
      fe_from_const(x, kGx);
      fe_from_const(y, kGy);
    }
    kok[base + g] = ok ? 1u : 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) kzq[(size_t)i * kC + base + g] = i == 0 ? 1u : 0u;   // u = 1: the chain runs on E
    u32* p = kqt + (size_t)(base + g) * L::NT * L::EW;
#pragma unroll
    for (int i = 0; i < 8; ++i) { p[i] = x.v[i]; p[8 + i] = y.v[i]; }
    gej29 q;
    f29_from_words(q.x, x.v);
    f29_from_words(q.y, y.v);
    f29_set_u32(q.z, 1);
#pragma unroll 1
    for (int grp = 1; grp < NG; ++grp) {
#pragma unroll 1
      for (int k = L::bit(grp - 1); k < L::bit(grp); ++k) gej29x_double(q, q);
      u32 xw[8], yw[8];
      f29_to_words(xw, q.x);
      f29_to_words(yw, q.y);
      u32* t = kqt2 + (size_t)((base + g) * (NG - 1) + (grp - 1)) * L::NT * L::EW;
#pragma unroll
      for (int i = 0; i < 8; ++i) { t[i] = xw[i]; t[8 + i] = yw[i]; }
      store_f29(kzq2 + (size_t)(grp - 1) * 8 * kC, kC, base + g, q.z);
    }
    return;
  }
#else
  fe x;
  load_fe(x, in_x, C, g);
  fe29 x29, c;
  {
    fe29 seven;
    f29_from_words(x29, x.v);
    f29x_sqr(c, x29);
    f29x_mul(c, c, x29);
    f29_set_u32(seven, 7);
    f29_add(c, c, seven);                   // c = x^3 + 7 (magnitude 2)
  }
  if (root) {
    const u32 pre = in_pfx[g];
    bool ok = (pre & 0xFEu) == 0x02u;
    {                                       // x < p  (btcec: "pubkey X parameter is >= to P")
      u32 br = 0, d;
#pragma unroll
      for (int i = 0; i < 8; ++i) d = __builtin_subc(x.v[i], kP[i], br, &br);
      (void)d;
      ok &= (br != 0);
    }
    fe29 y29, y2;
    f29x_sqrt_candidate(y29, c);            // y = c^((p+1)/4)
    f29x_sqr(y2, y29);
    ok &= f29_equal(y2, c);                 // "invalid square root"
    fe y;
    f29_to_words(y.v, y29);                 // canonical
    if ((y.v[0] & 1u) != (pre & 1u)) fe_neg(y, y);   // the prefix's parity (y != 0 always)
    fe_normalize(y);
    kok[base + g] = ok ? 1u : 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) kzq[(size_t)i * kC + base + g] = y.v[i];   // u, read by the table build
    return;
  }
  auto park = [](u32* tab, u32 row, const u32* xw, const u32* yw) {
    u32* p = tab + (size_t)row * L::NT * L::EW;
#pragma unroll
    for (int i = 0; i < 8; ++i) { p[i] = xw[i]; p[8 + i] = yw[i]; }
  };
  gej29 q;
  f29x_mul(q.x, c, x29);                    // Q' = (c x, c^2)
  f29x_sqr(q.y, c);
  f29_set_u32(q.z, 1);
  {
    u32 xw[8], yw[8];
    f29_to_words(xw, q.x);
    f29_to_words(yw, q.y);
    f29_from_words(q.x, xw);
    f29_from_words(q.y, yw);
    park(kqt, base + g, xw, yw);
  }
#pragma unroll 1
  for (int grp = 1; grp < NG; ++grp) {
#pragma unroll 1
    for (int k = L::bit(grp - 1); k < L::bit(grp); ++k) gej29x_double(q, q);  // Y never 0: no 2-torsion on E' or its twist
    u32 xw[8], yw[8];
    f29_to_words(xw, q.x);
    f29_to_words(yw, q.y);
    park(kqt2, (base + g) * (NG - 1) + (grp - 1), xw, yw);
    store_f29(kzq2 + (size_t)(grp - 1) * 8 * kC, kC, base + g, q.z);
  }
#endif
}

// k_keys_tables (lane L = 4 key + group, the four groups of a key in adjacent
// lanes of one wave): the group's table from its parked base point (X, Y)
// taken as affine -- the co-Z formulas never read the curve constant, so this
// is the table of the point on the isomorphic curve y^2 = x^3 + 7 Z^6, i.e.
// of the true point on table Z  E = Z_15 * Z.  The four lanes trade their E
// (lane shuffles) right after the forward pass, and the back-propagation that
// puts every entry on Z_15 also applies rho = the product of the other three
// E's: all four tables end on the common Z = E_0 E_1 E_2 E_3, so ONE
// accumulator can take entries of every group (k_ecmult_k4) -- no inversion
// and no extra pass over the tables.  Same co-Z steps as build_q_table.
// qr: Z-ratio scratch rows of stride C4 >= 4 n.  qe (may be null): rows of
// stride C4 for the forward pass's entries -- written and read back
// coalesced, so each table entry is written once, by the back-propagation
// (null: the entries go through the table itself: lanes 1,280 B apart write
// 80 B each, twice, and read them back in between).
// QW: 5 (k4, 16 entries per table) or 6 (the grouped route's k6, 32 entries).
// (four waves per SIMD: the launch is 4 waves per SIMD for 65,536 keys, so a
// fifth VGPR bank's worth would leave a third of a round as tail)
#ifndef GV_KEYS_TABLES_W4
#define GV_KEYS_TABLES_W4 1
#endif
#if GV_KEYS_TABLES_W4
#define GV_KEYS_TABLES_ATTR __attribute__((amdgpu_waves_per_eu(4)))
#else
#define GV_KEYS_TABLES_ATTR GV_FRONT_ATTR
#endif
template <int QW>
__global__ __launch_bounds__(256) GV_KEYS_TABLES_ATTR void k_keys_tables(u32 n, u32 C4, u32 base, u32* kqt, u32* kzq, u32 kC, u32* kqt2,
                                                      u32* kzq2, u32* qr, u32* qe) {
  constexpr int NT = KLayout<QW, 4>::NT;
  const u32 L = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 key = L >> 2, grp = L & 3u;
  if (key >= n) return;                     // whole quads only: shuffles stay inside live quads
  u32* tab = grp == 0u ? kqt : kqt2;
  const u32 row = grp == 0u ? base + key : (base + key) * GV_KEY2_TABLES + (grp - 1u);
  auto put = [&](int e, const fe29& x, const fe29& y) {
    if (qe) {
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        qe[((size_t)e * 18 + i) * C4 + L] = x.n[i];
        qe[((size_t)e * 18 + 9 + i) * C4 + L] = y.n[i];
      }
    } else {
      store_qent29<NT>(tab, row, e, x, y);
    }
  };
  auto get = [&](int e, fe29& x, fe29& y) {
    if (qe) {
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        x.n[i] = qe[((size_t)e * 18 + i) * C4 + L];
        y.n[i] = qe[((size_t)e * 18 + 9 + i) * C4 + L];
      }
    } else {
      load_qent29<NT>(x, y, tab, row, (u32)e);
    }
  };
  u32* zrow = grp == 0u ? kzq : kzq2 + (size_t)(grp - 1u) * 8 * kC;
  fe29 qx, qy, X1, Y1, X2, Y2, t, u, prod;
  {
    const u32* p = tab + (size_t)row * NT * GV_QENT_WORDS;
    u32 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = p[i];
    f29_from_words(qx, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = p[8 + i];
    f29_from_words(qy, w);
  }
  {
    // co-Z doubling of (qx, qy): Z1 = 2y, 2Q = (M^2 - 2S, M(S - X) - 8y^4),
    // Q' = (S, 8y^4) with S = 4xy^2, M = 3x^2.
    fe29 B, E, Lq, M;
    f29x_sqr(B, qx);
    f29x_sqr(E, qy);
    f29x_sqr(Lq, E);
    f29_add(t, qx, E);
    f29x_sqr(t, t);
    f29_sub<1>(t, t, B);
    f29_sub_norm<1>(t, t, Lq);
    f29_shl_norm<1>(X1, t);
    f29_mul3_norm(M, B);
    f29x_sqr(t, M);
    f29_add(u, X1, X1);
    f29_sub_norm<2>(X2, t, u);
    f29_shl_norm<3>(Y1, Lq);
    f29_sub<1>(t, X1, X2);
    f29x_mul(t, M, t);
    f29_sub_norm<1>(Y2, t, Y1);
  }
  put(0, X1, Y1);                           // 1*Q on Z1
  put(1, X2, Y2);                           // 2*Q on Z1
  f29_add(prod, qy, qy);                    // Z1 = 2y; times every ratio below -> Z_15
#pragma unroll 1
  for (int m = 2; m < NT; ++m) {            // (Q', mQ) -> ((m+1)Q, Q'')
    fe29 h, rr, c, w1, w2, d, a1;
    f29_sub_norm<1>(h, X1, X2);
    store_ratio29(qr, C4, L, m - 2, h);     // Z_m / Z_{m-1}
    f29x_mul(prod, prod, h);
    f29_sub_norm<1>(rr, Y1, Y2);
    f29x_sqr(c, h);
    f29x_mul(w1, X1, c);
    f29x_mul(w2, X2, c);
    f29x_sqr(d, rr);
    f29_sub<1>(t, w1, w2);
    f29x_mul(a1, Y1, t);
    f29_add(u, w1, w2);
    f29_sub_norm<2>(X2, d, u);
    f29_sub<1>(t, w1, X2);
    f29x_mul(t, rr, t);
    f29_sub_norm<1>(Y2, t, a1);
    X1 = w1;
    Y1 = a1;
    if (m + 1 < NT) put(m, X2, Y2);         // the last entry waits for rho
  }
  // E = Z_15 (times the parked Jacobian Z for groups 1..3, and u: the chain
  // ran on E', k_keys_chain); the quad's others
  if (grp) {
    fe29 z;
    load_f29(z, zrow, kC, base + key);
    f29x_mul(prod, prod, z);
  }
  {
    fe29 u;
    load_f29(u, kzq, kC, base + key);       // read by all four lanes before lane 0 writes zc there
    f29x_mul(prod, prod, u);
  }
  fe29 e1, e2, e3;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    e1.n[i] = (u32)__shfl_xor((int)prod.n[i], 1);
    e2.n[i] = (u32)__shfl_xor((int)prod.n[i], 2);
    e3.n[i] = (u32)__shfl_xor((int)prod.n[i], 3);
  }
  fe29 acc, zc;
  f29x_mul(acc, e1, e2);
  f29x_mul(acc, acc, e3);                    // rho
  f29x_mul(zc, acc, prod);                   // the common Z
  {
    fe29 a2, a3;                            // entry 16 (on Z_15): times rho^2, rho^3
    f29x_sqr(a2, acc);
    f29x_mul(a3, a2, acc);
    f29x_mul(X2, X2, a2);
    f29x_mul(Y2, Y2, a3);
    store_qent29<NT>(tab, row, NT - 1, X2, Y2);
  }
  // entry m (index m-1) on Z_{m-1} (m >= 2; entries 1, 2 on Z_1): times
  // rho * Z_15 / Z_{m-1}.  GV_KEYS_PREFETCH: the next iteration's ratio and
  // entry are loaded at the top of this one, so their latency hides under
  // this iteration's products (the loop is otherwise load-latency bound).
#if GV_KEYS_PREFETCH
  fe29 nr, nx, ny;
  if (NT - 1 >= 2) load_ratio29(nr, qr, C4, L, NT - 3);
  get(NT - 2, nx, ny);
#pragma unroll 1
  for (int m = NT - 1; m >= 1; --m) {
    fe29 x = nx, y = ny, ratio = nr;
    if (m >= 2) {                             // prefetch for m - 1
      if (m - 1 >= 2) load_ratio29(nr, qr, C4, L, m - 3);
      get(m - 2, nx, ny);
    }
    if (m >= 2) f29x_mul(acc, acc, ratio);
    fe29 a2, a3;
    f29x_sqr(a2, acc);
    f29x_mul(a3, a2, acc);
    f29x_mul(x, x, a2);
    f29x_mul(y, y, a3);
    store_qent29<NT>(tab, row, m - 1, x, y);
  }
#else
#pragma unroll 1
  for (int m = NT - 1; m >= 1; --m) {
    if (m >= 2) {
      fe29 ratio;
      load_ratio29(ratio, qr, C4, L, m - 2);
      f29x_mul(acc, acc, ratio);
    }
    fe29 x, y, a2, a3;
    f29x_sqr(a2, acc);
    f29x_mul(a3, a2, acc);
    get(m - 1, x, y);
    f29x_mul(x, x, a2);
    f29x_mul(y, y, a3);
    store_qent29<NT>(tab, row, m - 1, x, y);
  }
#endif
  store_f29(zrow, kC, base + key, zc);
}


// k_keys_fwd (lane L = NG key + group): the group's table from its parked base
// point (X, Y) taken as affine -- the co-Z formulas never read the curve
// constant, so this is the table of the point on the isomorphic curve
// y^2 = x^3 + 7 Z^6, i.e. of the true point on table Z  E = Z_last * Z.
// Forward pass only (co-Z doubling, then NT - 2 co-Z additions, Meloni's
// ZADDU: (Q', mQ) -> ((m+1) Q, Q'') for 4M + 2S, the new Z never formed --
// only the ratio X1 - X2 is kept): entry m - 1 (= m Q) lands on Z_{m-1}; the
// ratios go to the SoA rows qr (stride CL), the entries to the coalesced rows
// qe (or, qe null, the table itself: lanes a row apart writing 80 B each), E
// to the rows er.  No exceptional case: X(Q') == X(mQ) would need
// mQ == +-Q, i.e. n | m -+ 1, for 2 <= m <= NT - 1.
template <int QW, int NG>
GV_DEV void keys_put(u32* qe, u32 CL, u32 L, u32* tab, u32 row, int e, const fe29& x, const fe29& y) {
  if (qe) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      qe[((size_t)e * 18 + i) * CL + L] = x.n[i];
      qe[((size_t)e * 18 + 9 + i) * CL + L] = y.n[i];
    }
  } else {
    store_qent29<KLayout<QW, NG>::NT, KLayout<QW, NG>::EW>(tab, row, e, x, y);
  }
}
template <int QW, int NG>
GV_DEV void keys_get(const u32* qe, u32 CL, u32 L, const u32* tab, u32 row, int e, fe29& x, fe29& y) {
  if (qe) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      x.n[i] = qe[((size_t)e * 18 + i) * CL + L];
      y.n[i] = qe[((size_t)e * 18 + 9 + i) * CL + L];
    }
  } else {
    load_qent29<KLayout<QW, NG>::NT, KLayout<QW, NG>::EW>(x, y, tab, row, (u32)e);
  }
}

template <int QW, int NG>
__global__ __launch_bounds__(256) GV_FRONT_ATTR void k_keys_fwd(u32 n, u32 CL, u32 base, u32* kqt, u32 kC, u32* kqt2,
                                                   const u32* kzq2, u32* qr, u32* qe, u32* er, const u32* kzq) {
  constexpr int NT = KLayout<QW, NG>::NT;
  const u32 L = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 key = L / NG, grp = L % NG;
  if (key >= n) return;
  u32* tab = grp == 0u ? kqt : kqt2;
  const u32 row = grp == 0u ? base + key : (base + key) * (NG - 1) + (grp - 1u);
  fe29 qx, qy, X1, Y1, X2, Y2, t, u, prod;
  {
    const u32* p = tab + (size_t)row * NT * KLayout<QW, NG>::EW;
    u32 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = p[i];
    f29_from_words(qx, w);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = p[8 + i];
    f29_from_words(qy, w);
  }
  {
    // co-Z doubling of (qx, qy): Z1 = 2y, 2Q = (M^2 - 2S, M(S - X) - 8y^4),
    // Q' = (S, 8y^4) with S = 4xy^2, M = 3x^2.
    fe29 B, E, Lq, M;
    f29x_sqr(B, qx);
    f29x_sqr(E, qy);
    f29x_sqr(Lq, E);
    f29_add(t, qx, E);
    f29x_sqr(t, t);
    f29_sub<1>(t, t, B);
    f29_sub_norm<1>(t, t, Lq);
    f29_shl_norm<1>(X1, t);
    f29_mul3_norm(M, B);
    f29x_sqr(t, M);
    f29_add(u, X1, X1);
    f29_sub_norm<2>(X2, t, u);
    f29_shl_norm<3>(Y1, Lq);
    f29_sub<1>(t, X1, X2);
    f29x_mul(t, M, t);
    f29_sub_norm<1>(Y2, t, Y1);
  }
  keys_put<QW, NG>(qe, CL, L, tab, row, 0, X1, Y1);    // 1*Q on Z1
  keys_put<QW, NG>(qe, CL, L, tab, row, 1, X2, Y2);    // 2*Q on Z1
  f29_add(prod, qy, qy);                                 // Z1 = 2y; times every ratio below -> Z_last
#pragma unroll 1
  for (int m = 2; m < NT; ++m) {                         // (Q', mQ) -> ((m+1)Q, Q'')
    fe29 h, rr, c, w1, w2, d, a1;
    f29_sub_norm<1>(h, X1, X2);
    store_ratio29(qr, CL, L, m - 2, h);                  // Z_m / Z_{m-1}
    f29x_mul(prod, prod, h);
    f29_sub_norm<1>(rr, Y1, Y2);
    f29x_sqr(c, h);
    f29x_mul(w1, X1, c);
    f29x_mul(w2, X2, c);
    f29x_sqr(d, rr);
    f29_sub<1>(t, w1, w2);
    f29x_mul(a1, Y1, t);
    f29_add(u, w1, w2);
    f29_sub_norm<2>(X2, d, u);
    f29_sub<1>(t, w1, X2);
    f29x_mul(t, rr, t);
    f29_sub_norm<1>(Y2, t, a1);
    X1 = w1;
    Y1 = a1;
    keys_put<QW, NG>(qe, CL, L, tab, row, m, X2, Y2);    // (m+1)*Q on Z_m
  }
  // E = Z_last (times the parked Jacobian Z for groups 1.., and u: the chain
  // ran on E', k_keys_chain; k_keys_back overwrites kzq only in a later launch)
  if (grp) {
    fe29 z;
    load_f29(z, kzq2 + (size_t)(grp - 1u) * 8 * kC, kC, base + key);
    f29x_mul(prod, prod, z);
  }
  {
    fe29 u;
    load_f29(u, kzq, kC, base + key);
    f29x_mul(prod, prod, u);
  }
  store_ratio29(er, CL, L, 0, prod);
}

// k_keys_back (lane L = NG key + group): rho = the product of the OTHER
// groups' E (read from er), so every table lands on the key's common Z =
// E_0 ... E_{NG-1} -- ONE accumulator takes entries of every group, with no
// inversion -- then the back-propagation: entry m - 1 (on Z_{m-1}) times
// (rho Z_last / Z_{m-1})^2 and ^3, each table entry written once.
template <int QW, int NG>
__global__ __launch_bounds__(256) GV_FRONT_ATTR void k_keys_back(u32 n, u32 CL, u32 base, u32* kqt, u32* kzq, u32 kC,
                                                    u32* kqt2, u32* kzq2, const u32* qr, const u32* qe,
                                                    const u32* er) {
  constexpr int NT = KLayout<QW, NG>::NT;
  const u32 L = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 key = L / NG, grp = L % NG;
  if (key >= n) return;
  u32* tab = grp == 0u ? kqt : kqt2;
  const u32 row = grp == 0u ? base + key : (base + key) * (NG - 1) + (grp - 1u);
  u32* zrow = grp == 0u ? kzq : kzq2 + (size_t)(grp - 1u) * 8 * kC;
  fe29 acc, zc, own;
  bool first = true;
#pragma unroll 1
  for (u32 j = 0; j < (u32)NG; ++j) {
    fe29 e;
    load_ratio29(e, er, CL, key * NG + j, 0);
    if (j == grp) { own = e; continue; }
    if (first) acc = e;
    else f29x_mul(acc, acc, e);
    first = false;
  }
  f29x_mul(zc, acc, own);                                // the common Z
  // entry m - 1 on Z_{m-1} (m >= 2; entries 1, 2 on Z_1): times rho Z_last / Z_{m-1}
  // (GV_KEYS_PREFETCH: the next iteration's loads issued at the top, as k_keys_tables)
#if GV_KEYS_PREFETCH
  fe29 nr, nx, ny;
  keys_get<QW, NG>(qe, CL, L, tab, row, NT - 1, nx, ny);
#pragma unroll 1
  for (int m = NT; m >= 1; --m) {
    fe29 x = nx, y = ny, ratio = nr;
    if (m >= 2) {                                        // prefetch for m - 1
      if (m - 1 >= 2) load_ratio29(nr, qr, CL, L, m - 3);
      keys_get<QW, NG>(qe, CL, L, tab, row, m - 2, nx, ny);
    }
    if (m >= 2 && m < NT) f29x_mul(acc, acc, ratio);
    fe29 a2, a3;
    f29x_sqr(a2, acc);
    f29x_mul(a3, a2, acc);
    f29x_mul(x, x, a2);
    f29x_mul(y, y, a3);
    store_qent29<NT, KLayout<QW, NG>::EW>(tab, row, m - 1, x, y);
  }
#else
#pragma unroll 1
  for (int m = NT; m >= 1; --m) {
    if (m >= 2 && m < NT) {
      fe29 ratio;
      load_ratio29(ratio, qr, CL, L, m - 2);
      f29x_mul(acc, acc, ratio);
    }
    fe29 x, y, a2, a3;
    f29x_sqr(a2, acc);
    f29x_mul(a3, a2, acc);
    keys_get<QW, NG>(qe, CL, L, tab, row, m - 1, x, y);
    f29x_mul(x, x, a2);
    f29x_mul(y, y, a3);
    store_qent29<NT, KLayout<QW, NG>::EW>(tab, row, m - 1, x, y);
  }
#endif
  store_f29(zrow, kC, base + key, zc);
}

// Affine 2^35 G, 2^70 G, 2^100 G (16 words each) for the keyed ladder's G
// tables; thread t = group - 1.  Once per device.
__global__ void k_gen_gbase(u32* out) {
  const int t = threadIdx.x;
  if (t >= GV_KEY2_TABLES) return;
  const int* grp_bit = kLGrpBit;
  fe gx, gy;
  fe_from_const(gx, kGx);
  fe_from_const(gy, kGy);
  gej29 p;
  f29_from_words(p.x, gx.v);
  f29_from_words(p.y, gy.v);
  f29_set_u32(p.z, 1);
  for (int k = 0; k < grp_bit[t + 1]; ++k) gej29_double(p, p);
  fe x8, y8;
  gej29_to_affine_words(x8, y8, p);
#pragma unroll
  for (int i = 0; i < 8; ++i) { out[t * 16 + i] = x8.v[i]; out[t * 16 + 8 + i] = y8.v[i]; }
}

// Affine 2^o G (16 words each) for the full-scalar G tables' offsets o =
// kGFOff[t] (K6: the 6-bit-window ladders' tables, o = 24 t).
__constant__ const int kGFOff[GV_GF_NTAB] = {0, 45, 100, 145, 195, 220};
template <bool K6 = false>
__global__ void k_gen_gbasef(u32* out) {
  const int t = threadIdx.x;
  if (t >= (K6 ? GV_K6_GNTAB : GV_GF_NTAB)) return;
  const int off = K6 ? GV_K6_GW * t : kGFOff[t];
  fe gx, gy;
  fe_from_const(gx, kGx);
  fe_from_const(gy, kGy);
  gej29 p;
  f29_from_words(p.x, gx.v);
  f29_from_words(p.y, gy.v);
  f29_set_u32(p.z, 1);
  for (int k = 0; k < off; ++k) gej29_double(p, p);
  fe x8, y8;
  gej29_to_affine_words(x8, y8, p);
#pragma unroll
  for (int i = 0; i < 8; ++i) { out[t * 16 + i] = x8.v[i]; out[t * 16 + 8 + i] = y8.v[i]; }
}

// glat: per group, the multiples m = 1..16 of 2^(bit) G and 2^(bit) lambda G,
// affine; thread t = (group, part, m - 1).  Once per context.
__global__ void k_gen_glat(u32* glat) {
  const int t = threadIdx.x;
  if (t >= GV_LGRP * 2 * GV_QTAB_N) return;
  const int grp = t >> 5, part = (t >> 4) & 1, m = (t & 15) + 1;
  fe gx, gy;
  fe_from_const(gx, kGx);
  fe_from_const(gy, kGy);
  gej29 p;
  f29_from_words(p.x, gx.v);
  f29_from_words(p.y, gy.v);
  f29_set_u32(p.z, 1);
  if (part) {
    fe b8;
    fe29 beta;
    fe_from_const(b8, kBeta);
    f29_from_words(beta, b8.v);
    f29_mul(p.x, p.x, beta);                // lambda G = (beta x, y)
  }
  for (int k = 0; k < kLGrpBit[grp]; ++k) gej29_double(p, p);
  gej29 acc;
  bool inf = true;
  for (int b = 4; b >= 0; --b) {
    if (!inf) gej29_double(acc, acc);
    if ((m >> b) & 1) gej29_add_gej(acc, inf, acc, inf, p, false);
  }
  fe x8, y8;
  gej29_to_affine_words(x8, y8, acc);
  store_qent(glat, grp * 2 + part, m - 1, x8, y8);
}

// ------------------------------------------------------------ k_keys_point
// Key-arena readback (gv_keys_point): the affine point 1*Q of slot slots[g]
// from its table entry and shared Z (x = X / Z^2, y = Y / Z^3), as 64 bytes
// x || y big-endian, and the slot's ParsePubKey verdict.
__global__ __launch_bounds__(256) void k_keys_point(u32 n, const u32* slots, const u32* kqt, const u32* kzq,
                                                     u32 kC, const u32* kok, u32 kcount, uint8_t* out_xy,
                                                     uint8_t* out_ok) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const u32 sl = slots[g];
  uint8_t* o = out_xy + (size_t)g * 64;
  if (sl >= kcount) {
    for (int i = 0; i < 64; ++i) o[i] = 0;
    out_ok[g] = 0;
    return;
  }
  fe29 x, y, z, zi, z2, z3;
  load_qent29(x, y, kqt, sl, 0);
  load_f29(z, kzq, kC, sl);
  f29_inv(zi, z);
  f29_sqr(z2, zi);
  f29_mul(z3, z2, zi);
  f29_mul(x, x, z2);
  f29_mul(y, y, z3);
  u32 wx[8], wy[8];
  f29_to_words(wx, x);
  f29_to_words(wy, y);
  for (int i = 0; i < 8; ++i)
    for (int b = 0; b < 4; ++b) {
      o[4 * (7 - i) + b] = (uint8_t)(wx[i] >> (24 - 8 * b));
      o[32 + 4 * (7 - i) + b] = (uint8_t)(wy[i] >> (24 - 8 * b));
    }
  out_ok[g] = kok[sl] ? 1 : 0;
}

// ------------------------------------------------------------------ k_ecmult
// acc <- acc + (x, y) where (x, y) is affine on the accumulator's curve
// (zinv == nullptr: Q-table entry) or an affine point of the real curve to be
// lifted by zinv (G-table entry).  An infinite accumulator takes the point.
// x magnitude 1, y magnitude <= 2 (a negated entry), zinv magnitude 1.
// GV_FUSED: the ladder on the fused product engine (secp_group29x.cuh):
// subtractions and small multiples folded into the product chains (same
// results, fewer instructions per verify).  0 = the secp_group29.cuh formulas.
#ifndef GV_FUSED
#define GV_FUSED 1
#endif
GV_DEV void add_entry(gej29& acc, bool& inf, const fe29& x, const fe29& y, const fe29* zinv) {
#if GV_FUSED
  if (inf) {                                    // acc takes the entry, Z = 1
    if (zinv) {                                 // wave-uniform
      fe29 z2, z3;
      f29x_sqr(z2, *zinv);
      f29x_mul(acc.x, x, z2);
      f29x_mul(z3, z2, *zinv);
      f29x_mul(acc.y, y, z3);
    } else {
      acc.x = x;
      f29_norm(acc.y, y);                       // a negated entry has magnitude 2
    }
    f29_set_u32(acc.z, 1);
    inf = false;
    return;
  }
  fe29 az;
  if (zinv) f29x_mul(az, acc.z, *zinv);         // 1
  else az = acc.z;                              // <= 2
  gej29x_add_scaled(acc, inf, x, y, az);
#else
  fe29 az;
  if (zinv) {                                   // wave-uniform
    if (inf) az = *zinv;
    else f29_mul(az, acc.z, *zinv);             // 1
  } else {
    if (inf) f29_set_u32(az, 1);
    else az = acc.z;                            // <= 2
  }
  fe29 z2, u2, s2;
  f29_sqr(z2, az);
#if GV_ILP
  {
    fe29 o[2];
    const fe29 xa[2] = {x, z2}, ya[2] = {z2, az};
    f29_multi<false, false>(o, xa, ya);
    u2 = o[0]; z2 = o[1];
  }
#else
  f29_mul(u2, x, z2);
  f29_mul(z2, z2, az);
#endif
  f29_mul(s2, y, z2);                           // 2 x 1
  if (inf) {
    acc.x = u2;
    acc.y = s2;
    f29_set_u32(acc.z, 1);
    inf = false;
    return;
  }
  gej29_add_tail(acc, inf, u2, s2);
#endif
}

// Final check of a ladder: R = (X, Y, Z*zq) on the real curve; x(R) mod n ==
// r, inversion-free (X == r Z^2, or (r + n) Z^2 when r < p - n); accept
// bitmap by ballot.
// framed: acc is already on the real curve (Z as is; zq unused).
GV_DEV void ecmult_finish(const gej29& acc, bool inf, const fe29& zq, const u32* flags, const u32* in_r,
                          uint64_t* bits, u32 n, u32 C, u32 g, bool framed = false) {
  const u32 fl = flags[g];
  bool ok = (fl & 1u) && !inf;
  fe29 zr, zz, rf, t;
  if (framed) zr = acc.z;
  else f29_mul(zr, acc.z, zq);
  f29_sqr(zz, zr);
  u32 rw[8], X[8], tw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) rw[i] = in_r[(size_t)i * C + g];
  f29_from_words(rf, rw);
  f29_mul(t, rf, zz);
  f29_to_words(X, acc.x);
  f29_to_words(tw, t);
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) eq &= (X[i] == tw[i]);
  if (!eq && (fl & 2u)) {                   // R.x in [n, p): x mod n == r  <=>  x == r + n
    u32 rn[8];
    u32 c = 0;
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
  const uint64_t mask = __ballot(ok);
  if ((threadIdx.x & 63u) == 0 && (g >> 6) < ((n + 63u) >> 6)) bits[g >> 6] = mask;
}

// GV_STAMP (diagnostic builds only, `make ab NAME=stamp DEFS=-DGV_STAMP=1`):
// every wave of k_ecmult records its start and end shader clock
// (s_memtime) and 100 MHz real time (s_memrealtime) and where it ran (HW_ID,
// XCC_ID) into a buffer of its own that nothing else reads (gv_diag_stamps,
// tools/ecmult_stamps.py).  The product build has no stamp instruction.
#ifndef GV_STAMP
#define GV_STAMP 0
#endif
#if GV_STAMP
#define GV_STAMP_WAVES 65536
__device__ uint64_t g_stamps[2][GV_STAMP_WAVES * 6];
struct wave_stamp {
  uint64_t t0, r0;
  GV_DEV void begin() {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  GV_DEV void end(int which) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    u32 hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const u32 w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63u) == 0 && w < GV_STAMP_WAVES) {
      uint64_t* o = &g_stamps[which][(size_t)w * 6];
      o[0] = t0; o[1] = t1; o[2] = r0; o[3] = r1; o[4] = hw | ((uint64_t)xcc << 32); o[5] = blockIdx.x;
    }
  }
};
#define GV_STAMP_BEGIN wave_stamp stamp_; stamp_.begin();
#define GV_STAMP_END(k) stamp_.end(k);
#else
#define GV_STAMP_BEGIN
#define GV_STAMP_END(k)
#endif

// GV_ECMULT_WAVES: minimum waves per SIMD the register allocator must allow
// (0 = compiler's choice).
#ifndef GV_ECMULT_WAVES
#define GV_ECMULT_WAVES 0
#endif
#if GV_ECMULT_WAVES
#define GV_ECMULT_ATTR __attribute__((amdgpu_waves_per_eu(GV_ECMULT_WAVES)))
#else
#define GV_ECMULT_ATTR
#endif
// KEYED: the Q table and its Z come from key-arena row qidx[g] (zq rows of
// stride zC) instead of the lane's own row g (stride C).
// GF: G on the unsplit u1 from the full-scalar tables (gtab = gtabf; k_prep
// GF digits): window j (bit 25 j) is added at window position win from the
// table of offset kGFOff[kPGTab[j]] = 25 j - 5 win -- 11 G additions instead
// of the GLV schedule's 14 (the 26-window ladder spans bits 0..125, so the
// windows past it come from the 2^45, 2^100 and 2^145 tables).
__constant__ const int kPGWin[GV_QWIN][2] = {
    {0, -1}, {-1, -1}, {-1, -1}, {-1, -1}, {-1, -1}, {1, -1}, {-1, -1}, {-1, -1}, {-1, -1}, {-1, -1},
    {2, -1}, {-1, -1}, {-1, -1}, {-1, -1}, {-1, -1}, {3, 7},   {9, -1},  {-1, -1}, {-1, -1}, {-1, -1},
    {4, 8},  {6, 10},  {-1, -1}, {-1, -1}, {-1, -1}, {5, -1}};
__constant__ const int kPGTab[GV_GF_WIN] = {0, 0, 0, 0, 0, 0, 1, 2, 2, 3, 3};
template <bool KEYED, bool GF = false>
__global__ __launch_bounds__(256) GV_ECMULT_ATTR void k_ecmult(const u32* gtab, u32 n, u32 C, const u32* digits,
                                                 const u32* qt, const u32* zq_in, const u32* flags,
                                                 const u32* in_r, uint64_t* bits, const u32* qidx, u32 zC) {
  GV_STAMP_BEGIN
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 qi = KEYED ? qidx[g] : g;
  fe29 zq;
  load_f29(zq, zq_in, KEYED ? zC : C, qi);

  gej29 acc;
  f29_set_zero(acc.x); f29_set_zero(acc.y); f29_set_zero(acc.z);
  bool inf = true;

  // Strauss ladder: Q windows at bit 5*win, G windows at bit GV_GW*j = 5*(GV_GSTEP*j).
  // Slots per window: 0 = Q, 1 = lambda*Q (beta*x of the Q entry), and on G
  // windows 2 = G, 3 = lambda*G (second table).
#pragma unroll 1
  for (int win = GV_QWIN - 1; win >= 0; --win) {
    if (win != GV_QWIN - 1) {
#pragma unroll 1
#if GV_FUSED
      for (int d = 0; d < GV_QW; ++d) gej29x_double(acc, acc);
#else
      for (int d = 0; d < GV_QW; ++d) gej29_double(acc, acc);
#endif
    }
    const bool gwin = GF ? kPGWin[win][0] >= 0 : (win % GV_GSTEP) == 0;   // wave-uniform
    const u32 dq = digits[(size_t)win * C + g];
    u32 dg0 = 0u, dg1 = 0u;
    if (GF) {
      if (kPGWin[win][0] >= 0) dg0 = digits[(size_t)(GV_QWIN + kPGWin[win][0]) * C + g];
      if (kPGWin[win][1] >= 0) dg1 = digits[(size_t)(GV_QWIN + kPGWin[win][1]) * C + g];
    } else if (gwin) {
      const u32* grow = digits + (size_t)(GV_QWIN + 2 * (win / GV_GSTEP)) * C + g;
      dg0 = grow[0];
      dg1 = grow[C];
    }
    const int nslots = gwin ? 4 : 2;
#pragma unroll 1
    for (int slot = 0; slot < nslots; ++slot) {
      const int d = slot == 0 ? ((int)(dq << 16) >> 16) : slot == 1 ? ((int)dq >> 16)
                  : slot == 2 ? (int)dg0 : (int)dg1;
      if (d == 0) continue;
      const u32 e = (u32)((d < 0 ? -d : d) - 1);
      fe29 x, y;
      if (slot < 2) {
        load_qent29(x, y, qt, qi, e);
        if (slot == 1) {                           // lambda * P = (beta * x, y)
          fe29 beta;
          f29_from_const(beta, kBeta);
          f29_mul(x, x, beta);
        }
      } else if (GF) {                             // a missing second window has d == 0 (skipped above)
        load_gent29(x, y, gtab + (size_t)kPGTab[kPGWin[win][slot - 2]] * GV_GF_TAB_N * 16, e);
      } else {
        load_gent29(x, y, gtab + (slot == 3 ? (size_t)GV_GTAB_N * 16 : 0), e);
      }
      if (d < 0) f29_neg<1>(y, y);                 // 2
      add_entry(acc, inf, x, y, slot < 2 ? nullptr : &zq);
    }
  }

  ecmult_finish(acc, inf, zq, flags, in_r, bits, n, C, g);
  GV_STAMP_END(1)
}


// ------------------------------------------------------------- k_ecmult_k4
// Keyed batches: the key arena holds, per key, the tables of
// Q, 2^35 Q, 2^70 Q and 2^100 Q on ONE shared Z (k_keys_tables), and the
// device holds the 20-bit-window tables of G, 2^35 G, 2^70 G, 2^100 G (and
// lambda multiples).  Each 128-bit GLV half's 26 five-bit windows split into
// the groups [0,7), [7,14), [14,20), [20,26); window w of group k sits at
// local position w - w0(k) of a 35-bit ladder, so one accumulator takes every
// group's entry at that position: 6 x 5 = 30 doublings instead of 125, the
// same 52 Q + 14 G additions.  G window j (bit 20 j) is taken from the G
// table of the largest group offset <= 20 j at local position (20 j - b)/5.
static_assert(GV_GW == 20 && GV_QWIN == 26 && GV_LGRP == 4, "k_ecmult_k4 layout");
__constant__ const int kK4WStart[4] = {0, 7, 14, 20};
__constant__ const int kK4NWin[4] = {7, 7, 6, 6};
__constant__ const int kK4GWin[7][2] = {{0, 5}, {2, -1}, {4, -1}, {-1, -1}, {1, 6}, {3, -1}, {-1, -1}};
__constant__ const int kK4GGrp[7] = {0, 0, 1, 1, 2, 3, 3};
// GF (gv_kernels.h GV_GF_*): the G windows j at each position (up to four)
// and the table each reads (offset kGFOff[kGFTab[j]] = 25 j - 5 p)
__constant__ const int kGFWin[7][4] = {{0, 4, -1, -1}, {2, 6, 8, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1},
                                       {-1, -1, -1, -1}, {1, 5, -1, -1}, {3, 7, 9, 10}};
__constant__ const int kGFTab[GV_GF_WIN] = {0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5};

// GV_LAMFRAME (default 1): at each position the four groups' Q entries are
// added first, then the accumulator moves to lambda^2 (x -> beta^2 x), takes
// the lambda-Q entries' plain (x, y) -- lambda^2 A + T = lambda^2 (A + lambda T),
// lambda^3 = 1 -- and moves back (x -> beta x) before the G entries: two
// beta products per position instead of one per lambda-Q entry.  The same
// sum (lambda is a group automorphism, so the exceptional cases -- H == 0 --
// meet the same points); 0: beta x per lambda-Q entry.
#ifndef GV_LAMFRAME
#define GV_LAMFRAME 1
#endif
#ifndef GV_LAMREV
#define GV_LAMREV 1
#endif
// GF: gtab is the full-scalar G tables (gtabf), gtab4 unused.
template <bool GF>
__global__ __launch_bounds__(256) GV_ECMULT_ATTR void k_ecmult_k4(const u32* gtab, const u32* gtab4, u32 n, u32 C,
                                                        const u32* digits, const u32* kqt, const u32* kqt2,
                                                        const u32* kzq, const u32* flags, const u32* in_r,
                                                        uint64_t* bits, const u32* qidx, u32 kC) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 qi = qidx[g];
  fe29 zq;
  load_f29(zq, kzq, kC, qi);
  gej29 acc;
  f29_set_zero(acc.x); f29_set_zero(acc.y); f29_set_zero(acc.z);
  bool inf = true;
#pragma unroll 1
  for (int pos = 6; pos >= 0; --pos) {
    if (pos != 6) {
#pragma unroll 1
      for (int d = 0; d < GV_QW; ++d) gej29x_double(acc, acc);
    }
    // slots 0..7: (group, Q / lambda Q) -- LAMFRAME: Q of groups 0..3, then
    // lambda Q of groups 0..3 on lambda^2 (acc); 8..11: up to two G windows x
    // (G, lambda G) or (GF) up to four G windows
#pragma unroll 1
    for (int slot = 0; slot < 12; ++slot) {
      if (GV_LAMFRAME && (slot == 4 || slot == 8) && !inf) {
        fe29 c;                                            // into lambda^2 (acc) / back to acc
        f29_from_const(c, slot == 4 ? kBeta2 : kBeta);
        f29x_mul(acc.x, acc.x, c);
      }
      int d;
      const u32* tab;
      u32 row = 0;
      const bool isg = slot >= 8;
      const bool lam = GV_LAMFRAME ? slot >= 4 : (slot & 1) != 0;
      if (!isg) {
        // (lambda entries in reverse group order: group 3's row was read last)
        const int grp = GV_LAMFRAME ? (lam && GV_LAMREV ? 3 - (slot & 3) : (slot & 3)) : (slot >> 1);
        if (pos >= kK4NWin[grp]) continue;                 // wave-uniform
        const u32 dq = digits[(size_t)(kK4WStart[grp] + pos) * C + g];
        d = lam ? ((int)dq >> 16) : ((int)(dq << 16) >> 16);
        tab = grp == 0 ? kqt : kqt2;
        row = grp == 0 ? qi : qi * GV_KEY2_TABLES + (grp - 1);
      } else if (GF) {
        const int j = kGFWin[pos][slot - 8];
        if (j < 0) continue;                               // wave-uniform
        d = (int)digits[(size_t)(GV_QWIN + j) * C + g];
        tab = gtab + (size_t)kGFTab[j] * GV_GF_TAB_N * 16;
      } else {
        const int j = kK4GWin[pos][(slot - 8) >> 1];
        if (j < 0) continue;                               // wave-uniform
        d = (int)digits[(size_t)(GV_QWIN + 2 * j + (slot & 1)) * C + g];
        const int gg = kK4GGrp[j];
        tab = (gg == 0 ? gtab : gtab4 + (size_t)(gg - 1) * 2 * GV_GTAB_N * 16) +
              ((slot & 1) ? (size_t)GV_GTAB_N * 16 : 0);
      }
      if (d == 0) continue;
      const u32 e = (u32)((d < 0 ? -d : d) - 1);
      fe29 x, y;
      if (!isg) {
        load_qent29(x, y, tab, row, e);
        if (lam && !GV_LAMFRAME) {                         // lambda * P = (beta * x, y)
          fe29 beta;
          f29_from_const(beta, kBeta);
          f29x_mul(x, x, beta);
        }
      } else {
        load_gent29(x, y, tab, e);
      }
      if (d < 0) f29_neg<1>(y, y);                         // 2
      add_entry(acc, inf, x, y, isg ? &zq : nullptr);
    }
  }
  ecmult_finish(acc, inf, zq, flags, in_r, bits, n, C, g);
}

// ------------------------------------------------------------- k_ecmult_kn
// The 6-bit-window keyed ladders (gv_kernels.h GV_K6_*, KLayout<6, NG>): the
// key tables hold 32 multiples per group, so each 128-bit GLV half takes 22
// six-bit windows, split into NG groups; window w of group k is added at
// local position w - w0(k) of a P-position ladder: 6 (P - 1) doublings
// (NG = 4: 30; the resident arena's NG = 11: 6) and 44 Q additions (52 with
// 5-bit windows).  At each position the Q entries of groups 0.. go first,
// then the accumulator moves to lambda^2 (x -> beta^2 x), takes the
// lambda-Q entries of groups ..0 as plain (x, y) -- lambda^2 A + T =
// lambda^2 (A + lambda T) since lambda^3 = 1 -- and moves back (x -> beta x):
// two beta products per position.  G on the unsplit u1: its 11 signed 24-bit
// windows (window j at bit 24 j) are added after the last doubling from the
// 2^23-entry tables of 2^(24 j) G.  Same additions, final check and semantics
// as k_ecmult_k4 otherwise (lambda is a group automorphism, so every
// exceptional case -- H == 0 -- meets the same points).
// QW = GV_KW_QW (the arena's wide-window tables, GV_KW_*: 11 by default): 12
// eleven-bit windows per GLV half, in 12 groups (one position, no doublings)
// or 6 (two positions, 11 doublings), 1,024-entry tables, 24 Q additions.
// The group layout as constant tables (row 0: NG = 4, row 1: the arena's NG,
// row 2: the wide arena's NG) -- indexing them keeps the ladder's register
// allocation at that of k4
#define GV_KN_ROW(QW, NG, F) KLayout<QW, NG>::F(0), KLayout<QW, NG>::F(1), KLayout<QW, NG>::F(2), \
    KLayout<QW, NG>::F(3), KLayout<QW, NG>::F(4), KLayout<QW, NG>::F(5), KLayout<QW, NG>::F(6), \
    KLayout<QW, NG>::F(7), KLayout<QW, NG>::F(8), KLayout<QW, NG>::F(9), KLayout<QW, NG>::F(10), \
    KLayout<QW, NG>::F(11), KLayout<QW, NG>::F(12), KLayout<QW, NG>::F(13), KLayout<QW, NG>::F(14), \
    KLayout<QW, NG>::F(15), KLayout<QW, NG>::F(16), KLayout<QW, NG>::F(17), KLayout<QW, NG>::F(18)
// rows 4.. : the grouped route's 5-bit many-group layouts (GV_KG_NGS)
__constant__ const int kKnW0[8][19] = {
    {GV_KN_ROW(6, 4, w0)},
    {GV_KN_ROW(6, GV_KN_ARENA_NG, w0)},
    {GV_KN_ROW(GV_KW_QW, GV_KW_NG2, w0)},
    {GV_KN_ROW(GV_KW_QW, GV_KW_NG1, w0)},
    {GV_KN_ROW(GV_QW, 6, w0)},
    {GV_KN_ROW(GV_QW, 7, w0)},
    {GV_KN_ROW(GV_QW, 9, w0)},
    {GV_KN_ROW(GV_QW, 4, w0)}};
__constant__ const int kKnNW[8][19] = {
    {GV_KN_ROW(6, 4, nw)},
    {GV_KN_ROW(6, GV_KN_ARENA_NG, nw)},
    {GV_KN_ROW(GV_KW_QW, GV_KW_NG2, nw)},
    {GV_KN_ROW(GV_KW_QW, GV_KW_NG1, nw)},
    {GV_KN_ROW(GV_QW, 6, nw)},
    {GV_KN_ROW(GV_QW, 7, nw)},
    {GV_KN_ROW(GV_QW, 9, nw)},
    {GV_KN_ROW(GV_QW, 4, nw)}};
#undef GV_KN_ROW
static_assert(GV_KN_ARENA_NG <= 16 && GV_KW_NG1 <= 19, "layout table rows");

constexpr int kn_row(int qw, int ng) {
  return qw == 6 && ng == 4                    ? 0
         : qw == 6 && ng == GV_KN_ARENA_NG     ? 1
         : qw == GV_KW_QW && ng == GV_KW_NG2   ? 2
         : qw == GV_KW_QW && ng == GV_KW_NG1   ? 3
         : qw == GV_QW && ng == 6              ? 4
         : qw == GV_QW && ng == 7              ? 5
         : qw == GV_QW && ng == 9              ? 6
         : qw == GV_QW && ng == 4              ? 7
                                               : -1;
}
// GV_KN_GFRAME (default 1, round 6): after the last Q entry the accumulator
// moves from the key tables' Z onto the real curve (Z <- Z zq, one product),
// so the 11 G entries are added without the per-entry lift az = Z zq and the
// final check skips its Z zq: 11 products fewer per verify.  The same point
// and the same exceptional cases (the lift only rescaled the Jacobian
// representative).  0: every G entry lifted (rounds 4-5).
#ifndef GV_KN_GFRAME
#define GV_KN_GFRAME 1
#endif

// GV_KN_WAVES: the same bound for k_ecmult_kn alone (A/B: its gathers from the
// resident arena's large tables wait longer than k_ecmult_k4's)
#ifndef GV_KN_WAVES
#define GV_KN_ATTR GV_ECMULT_ATTR
#else
#define GV_KN_ATTR __attribute__((amdgpu_waves_per_eu(GV_KN_WAVES)))
#endif
// GV_KN_ZQ_LDS (round 6, the 5-bit kg ladders only): with the G frame
// change zq is read once, at the end; held in registers across the ladder it
// takes k_ecmult_kn<5, NG> to 160 VGPRs (3 waves per SIMD, 32 VGPRs left for a
// front kernel's wave), parked in LDS (9 KB per block) to 126: 4 waves per
// SIMD (kg4: C2 216 -> 222M/s alternated, profiles/r06/ab/ab3).  The arena's
// ladders keep zq in registers (kw at 133 VGPRs: 440 vs 428M/s with LDS).
#ifndef GV_KN_ZQ_LDS
#define GV_KN_ZQ_LDS 1
#endif
// GV_KN_PREFETCH (A/B, round 6): the slot loop runs one slot ahead -- slot
// s + 1's digit is read and its table entry's loads issued before slot s's
// addition, so the gather's latency hides under ~1.5k VALU of the addition
// instead of stalling the wave (the resident arena's wide tables are read
// from HBM: VALU busy 0.83 at round 5).  Same additions in the same order.
#ifndef GV_KN_PREFETCH
#define GV_KN_PREFETCH 0
#endif
// raw table-entry words in flight: Q entries (EW words), G entries (16 words)
template <int NT, int EW>
GV_DEV void fetch_qent(uint4* r, const u32* qt, u32 g, u32 j) {
  const uint4* p = (const uint4*)(qt + ((size_t)g * NT + j) * EW);
  r[0] = p[0]; r[1] = p[1]; r[2] = p[2]; r[3] = p[3];
  if constexpr (EW != 16) r[4] = p[4];
}
template <int EW>
GV_DEV void unpack_qent(fe29& x, fe29& y, const uint4* r) {
  if constexpr (EW == 16) {
    const u32 xw[8] = {r[0].x, r[0].y, r[0].z, r[0].w, r[1].x, r[1].y, r[1].z, r[1].w};
    const u32 yw[8] = {r[2].x, r[2].y, r[2].z, r[2].w, r[3].x, r[3].y, r[3].z, r[3].w};
    f29_from_words(x, xw);
    f29_from_words(y, yw);
  } else {
    x.n[0] = r[0].x; x.n[1] = r[0].y; x.n[2] = r[0].z; x.n[3] = r[0].w;
    x.n[4] = r[1].x; x.n[5] = r[1].y; x.n[6] = r[1].z; x.n[7] = r[1].w;
    x.n[8] = r[2].x; y.n[0] = r[2].y; y.n[1] = r[2].z; y.n[2] = r[2].w;
    y.n[3] = r[3].x; y.n[4] = r[3].y; y.n[5] = r[3].z; y.n[6] = r[3].w;
    y.n[7] = r[4].x; y.n[8] = r[4].y;
  }
}

template <int QW, int NG>
__global__ __launch_bounds__(256) GV_KN_ATTR void k_ecmult_kn(const u32* gtab6, u32 n, u32 C, const u32* digits,
                                                        const u32* kqt, const u32* kqt2, const u32* kzq,
                                                        const u32* flags, const u32* in_r, uint64_t* bits,
                                                        const u32* qidx, u32 kC) {
  using L = KLayout<QW, NG>;
  constexpr int T = kn_row(QW, NG);
  static_assert(T >= 0, "a layout row of kKnW0 / kKnNW");
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 qi = qidx[g];
  fe29 zq;
  load_f29(zq, kzq, kC, qi);
  constexpr bool ZL = GV_KN_ZQ_LDS && GV_KN_GFRAME && QW == GV_QW;
  __shared__ u32 zq_lds[ZL ? 9 : 1][256];        // ZL: zq parked in LDS until the frame change
  if constexpr (ZL) {
#pragma unroll
    for (int i = 0; i < 9; ++i) zq_lds[i][threadIdx.x] = zq.n[i];
  }
  gej29 acc;
  f29_set_zero(acc.x); f29_set_zero(acc.y); f29_set_zero(acc.z);
  bool inf = true;
#pragma unroll 1
  for (int pos = L::P - 1; pos >= 0; --pos) {
    if (pos != L::P - 1) {
#pragma unroll 1
      for (int d = 0; d < QW; ++d) gej29x_double(acc, acc);
    }
    // slots 0..NG-1: Q of groups 0..NG-1; NG..2NG-1: lambda Q of groups
    // NG-1..0 on the lambda^2 frame; then (position 0) the 11 G windows
    // (the wide-window ladders only: the others would pass 168 VGPRs, 2 waves)
    if constexpr (GV_KN_PREFETCH && QW == GV_KW_QW) {
    constexpr int NSLOT = 2 * NG + GV_K6_GWIN;
    // slot s's digit (0: nothing to add -- a window past the group's, or G
    // off position 0) and the issue of its entry's loads into r
    auto fetch = [&](int slot, uint4* r) -> int {
      if (slot >= 2 * NG) {
        if (pos != 0) return 0;
        const int j = slot - 2 * NG;
        const int d = (int)digits[(size_t)(L::QWIN + j) * C + g];
        if (d) {
          const uint4* p = (const uint4*)(gtab6 + (size_t)j * GV_K6_GTAB_N * 16 + (size_t)((d < 0 ? -d : d) - 1) * 16);
          r[0] = p[0]; r[1] = p[1]; r[2] = p[2]; r[3] = p[3];
        }
        return d;
      }
      const bool lam = slot >= NG;
      const int grp = lam ? 2 * NG - 1 - slot : slot;
      if (pos >= kKnNW[T][grp]) return 0;
      const u32 dq = digits[(size_t)(kKnW0[T][grp] + pos) * C + g];
      const int d = lam ? ((int)dq >> 16) : ((int)(dq << 16) >> 16);
      if (d) fetch_qent<L::NT, L::EW>(r, grp == 0 ? kqt : kqt2, grp == 0 ? qi : qi * (NG - 1) + (grp - 1),
                                        (u32)((d < 0 ? -d : d) - 1));
      return d;
    };
    uint4 rn[5];
    int dn = fetch(0, rn);
#pragma unroll 1
    for (int slot = 0; slot < NSLOT; ++slot) {
      uint4 rc[5] = {rn[0], rn[1], rn[2], rn[3], rn[4]};
      const int d = dn;
      if (slot + 1 < NSLOT) dn = fetch(slot + 1, rn);
      if ((slot == NG || slot == 2 * NG) && !inf) {
        fe29 c;                                            // into lambda^2 (acc) / back to acc
        f29_from_const(c, slot == NG ? kBeta2 : kBeta);
        f29x_mul(acc.x, acc.x, c);
      }
      if (slot >= 2 * NG && pos != 0) break;               // wave-uniform: G after the last doubling
      if (GV_KN_GFRAME && slot == 2 * NG && !inf) {
        fe29 z;
        if constexpr (ZL) {
#pragma unroll
          for (int i = 0; i < 9; ++i) zq.n[i] = zq_lds[i][threadIdx.x];
        }
        f29x_mul(z, acc.z, zq);
        acc.z = z;
      }
      if (d == 0) continue;
      const bool isg = slot >= 2 * NG;
      fe29 x, y;
      if (!isg) {
        unpack_qent<L::EW>(x, y, rc);
      } else {
        const u32 xw[8] = {rc[0].x, rc[0].y, rc[0].z, rc[0].w, rc[1].x, rc[1].y, rc[1].z, rc[1].w};
        const u32 yw[8] = {rc[2].x, rc[2].y, rc[2].z, rc[2].w, rc[3].x, rc[3].y, rc[3].z, rc[3].w};
        f29_from_words(x, xw);
        f29_from_words(y, yw);
      }
      if (d < 0) f29_neg<1>(y, y);                         // 2
      add_entry(acc, inf, x, y, isg && !GV_KN_GFRAME ? &zq : nullptr);
    }
    } else {
#pragma unroll 1
    for (int slot = 0; slot < 2 * NG + GV_K6_GWIN; ++slot) {
      if ((slot == NG || slot == 2 * NG) && !inf) {
        fe29 c;                                            // into lambda^2 (acc) / back to acc
        f29_from_const(c, slot == NG ? kBeta2 : kBeta);
        f29x_mul(acc.x, acc.x, c);
      }
      if (slot >= 2 * NG && pos != 0) break;               // wave-uniform: G after the last doubling
      if (GV_KN_GFRAME && slot == 2 * NG && !inf) {
        // onto the real curve: acc (X, Y, Z) on the tables' Z is the point
        // (X, Y, Z zq), so the G entries are added unlifted (az = Z) and the
        // final check reads Z as is
        fe29 z;
        if constexpr (ZL) {
#pragma unroll
          for (int i = 0; i < 9; ++i) zq.n[i] = zq_lds[i][threadIdx.x];
        }
        f29x_mul(z, acc.z, zq);
        acc.z = z;
      }
      int d;
      const u32* tab;
      u32 row = 0;
      const bool isg = slot >= 2 * NG;
      if (!isg) {
        const bool lam = slot >= NG;
        const int grp = lam ? 2 * NG - 1 - slot : slot;
        if (pos >= kKnNW[T][grp]) continue;                // wave-uniform
        const u32 dq = digits[(size_t)(kKnW0[T][grp] + pos) * C + g];
        d = lam ? ((int)dq >> 16) : ((int)(dq << 16) >> 16);
        tab = grp == 0 ? kqt : kqt2;
        row = grp == 0 ? qi : qi * (NG - 1) + (grp - 1);
      } else {
        const int j = slot - 2 * NG;
        d = (int)digits[(size_t)(L::QWIN + j) * C + g];
        tab = gtab6 + (size_t)j * GV_K6_GTAB_N * 16;
      }
      if (d == 0) continue;
      const u32 e = (u32)((d < 0 ? -d : d) - 1);
      fe29 x, y;
      if (!isg) load_qent29<L::NT, L::EW>(x, y, tab, row, e);
      else load_gent29(x, y, tab, e);
      if (d < 0) f29_neg<1>(y, y);                         // 2
      add_entry(acc, inf, x, y, isg && !GV_KN_GFRAME ? &zq : nullptr);
    }
    }
  }
  // GV_KN_GFRAME: acc is on the real curve (or infinite: rejected either way)
  ecmult_finish(acc, inf, zq, flags, in_r, bits, n, C, g, GV_KN_GFRAME != 0);
}

// ------------------------------------------------------------------- k_debug
// Test hook (gv_debug_op in the C-ABI): exercises one building block per lane
// so the GPU tests can pin field/scalar/GLV arithmetic against the oracle.
// in: 16 words per item (a = words 0..7, b = 8..15, little-endian limbs);
// out: 16 words per item.
__global__ void k_debug(int op, u32 n, const u32* in, u32* out) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = g < n;
  const u32 gi = live ? g : 0u;
  fe a, b, r;
#pragma unroll
  for (int i = 0; i < 8; ++i) { a.v[i] = in[gi * 16 + i]; b.v[i] = in[gi * 16 + 8 + i]; }
  u32 o[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) o[i] = 0;
  switch (op) {
    case 0: fe_mul(r, a, b); fe_normalize(r); break;
    case 1: fe_sqr(r, a); fe_normalize(r); break;
    case 2: fe_add(r, a, b); fe_normalize(r); break;
    case 3: fe_sub(r, a, b); fe_normalize(r); break;
    case 4: fe_inv(r, a); fe_normalize(r); break;
    case 5: fe_sqrt_candidate(r, a); fe_normalize(r); break;
    case 6: r = a; fe_normalize(r); break;
    case 7: { u32 t[16]; mul_256x256(t, a.v, b.v);
#pragma unroll
              for (int i = 0; i < 16; ++i) o[i] = t[i];
              r = a; break; }
    case 8: { sc_montmul(r.v, a.v, b.v); break; }
    case 9: { u32 k1[4], k2[4], n1, n2; glv_split(k1, n1, k2, n2, a.v);
#pragma unroll
              for (int i = 0; i < 4; ++i) { o[i] = k1[i]; o[4 + i] = k2[i]; }
              o[8] = n1; o[9] = n2; r = a; break; }
    case 10: { // batch inversion of a (plain form, nonzero) across the wave -> plain inverse
               // (the production path: radix-2^29 Montgomery, secp_sc29.cuh)
              u32 one[8] = {1u, 0, 0, 0, 0, 0, 0, 0};
              if (!live || u256_is_zero(a.v)) { for (int i = 0; i < 8; ++i) a.v[i] = one[i]; }
              sc29 x, xm, im, o1, pl;
              sc29_from_words(x, a.v); sc29_to_mont(xm, x); sc29_batch_inv_wave(im, xm);
              sc29_from_words(o1, one); sc29_mul(pl, im, o1); sc29_to_words(r.v, pl); break; }
    case 27: { // a^-1 mod n by divsteps (secp_modinv.cuh; the latency kernel's s^-1)
              s30_modinv(r.v, a.v, [](bool done) { return __all(done) != 0; }); break; }
    case 26: { // radix-2^29 Montgomery product a * b * 2^-261 mod n, canonical
              sc29 x, y, z; sc29_from_words(x, a.v); sc29_from_words(y, b.v); sc29_mul(z, x, y);
              sc29_to_words(r.v, z); break; }
    case 11: { // Jacobian double of affine (a, b), returned affine
              gej p; p.x = a; p.y = b; fe_set_u32(p.z, 1); gej_double(p, p);
              fe zi, z2, z3; fe_inv(zi, p.z); fe_sqr(z2, zi); fe_mul(z3, z2, zi);
              fe_mul(r, p.x, z2); fe_mul(p.y, p.y, z3); fe_normalize(r); fe_normalize(p.y);
#pragma unroll
              for (int i = 0; i < 8; ++i) o[8 + i] = p.y.v[i];
              break; }
    case 12: fe_shl<1>(r, a); fe_normalize(r); break;
    case 13: fe_shl<2>(r, a); fe_normalize(r); break;
    case 14: fe_shl<3>(r, a); fe_normalize(r); break;
    case 15: fe_mul3(r, a); fe_normalize(r); break;
    case 16: fe_sub_shl<1>(r, a, b); fe_normalize(r); break;
    case 17: fe_sub_shl<2>(r, a, b); fe_normalize(r); break;
    case 18: fe_sub_shl<3>(r, a, b); fe_normalize(r); break;
    // 9 x 29 layer (secp_fe29.cuh / secp_group29.cuh): words in, canonical words out
    case 19: case 20: case 21: case 22: case 23: case 25: {
      fe29 x, y, z;
      f29_from_words(x, a.v);
      f29_from_words(y, b.v);
      if (op == 19) f29_mul(z, x, y);
      else if (op == 20) f29_sqr(z, x);
      else if (op == 21) f29_sub_norm<1>(z, x, y);
      else if (op == 22) f29_inv(z, x);
      else if (op == 23) f29_sqrt_candidate(z, x);
      else { f29_sub_norm<1>(z, x, y); f29_set_u32(z, f29_is_zero_fast(z) ? 1u : 0u); }
      f29_to_words(r.v, z);
      break;
    }
    case 24: {  // Jacobian double of affine (a, b) on the 9 x 29 layer, returned affine
      gej29 q;
      f29_from_words(q.x, a.v); f29_from_words(q.y, b.v); f29_set_u32(q.z, 1);
      gej29_double(q, q);
      fe29 zi, z2, z3;
      f29_inv(zi, q.z); f29_sqr(z2, zi); f29_mul(z3, z2, zi);
      f29_mul(q.x, q.x, z2); f29_mul(q.y, q.y, z3);
      f29_to_words(r.v, q.x);
      u32 yw[8];
      f29_to_words(yw, q.y);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[8 + i] = yw[i];
      break;
    }
    default: r = a; break;
  }
  if (op != 7 && op != 9) {
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (op == 11 && false) ? 0u : r.v[i];
  }
  if (live) {
#pragma unroll
    for (int i = 0; i < 16; ++i) out[g * 16 + i] = o[i];
  }
}

}  // namespace gv

// ------------------------------------------------------------- host launchers
extern "C" {

hipError_t gvk_gen_gtable(uint32_t* gtab, hipStream_t st) {
  hipLaunchKernelGGL(gv::k_gen_gtable<GV_GTAB_N>, dim3((GV_GTAB_N + 63) / 64), dim3(64), 0, st, gtab,
                     (const uint32_t*)nullptr);
  return hipGetLastError();
}

hipError_t gvk_gen_gtable4(uint32_t* gtab4, uint32_t* base_scratch, hipStream_t st) {
  hipLaunchKernelGGL(gv::k_gen_gbase, dim3(1), dim3(64), 0, st, base_scratch);
  for (int k = 0; k < GV_KEY2_TABLES; ++k)
    hipLaunchKernelGGL(gv::k_gen_gtable<GV_GTAB_N>, dim3((GV_GTAB_N + 63) / 64), dim3(64), 0, st,
                       gtab4 + (size_t)k * 2 * GV_GTAB_N * 16, (const uint32_t*)(base_scratch + 16 * k));
  return hipGetLastError();
}

hipError_t gvk_gen_gtable6(uint32_t* gtab6, uint32_t* base_scratch, hipStream_t st) {
  hipLaunchKernelGGL(gv::k_gen_gbasef<true>, dim3(1), dim3(64), 0, st, base_scratch);
  const dim3 grd((GV_K6_GTAB_N + 255) / 256), blk(256);
  for (int k = 0; k < GV_K6_GNTAB; ++k)
    hipLaunchKernelGGL((gv::k_gen_gtable<GV_K6_GTAB_N, false>), grd, blk, 0, st, gtab6 + (size_t)k * GV_K6_GTAB_N * 16,
                       (const uint32_t*)(base_scratch + 16 * k));
  return hipGetLastError();
}

hipError_t gvk_gen_gtablef(uint32_t* gtabf, uint32_t* base_scratch, hipStream_t st) {
  hipLaunchKernelGGL(gv::k_gen_gbasef<false>, dim3(1), dim3(64), 0, st, base_scratch);
  const dim3 grd((GV_GF_TAB_N + 255) / 256), blk(256);
  for (int k = 0; k < GV_GF_NTAB; ++k)
    hipLaunchKernelGGL((gv::k_gen_gtable<GV_GF_TAB_N, false>), grd, blk, 0, st, gtabf + (size_t)k * GV_GF_TAB_N * 16,
                       (const uint32_t*)(base_scratch + 16 * k));
  return hipGetLastError();
}

hipError_t gvk_verify(const gvk_batch* b, hipStream_t st) {
  const uint32_t C = b->C;
  const dim3 blk(256), grd(C / 256);
  // key-ordered lanes (gv_sort.hip): keyed k4 batches with sort scratch
  const bool k6 = b->kslot && b->k6 && b->gtab6;
  const bool kw = k6 && b->kqw == 1 && (b->k6 == GV_KW_NG1 || b->k6 == GV_KW_NG2);   // the arena's wide-window tables
  const bool kg = k6 && b->kqw == 2;             // the grouped route's 5-bit many-group tables
  const bool gf = b->kslot && b->gtab4 && b->gtabf && !k6;   // k_ecmult_k4<true>
  const bool gfp = !b->kslot && b->gtabf;                     // per-item pub33: k_ecmult<false, true>
  const bool sorted = b->kslot && (b->gtab4 || k6) && b->srt.perm;
  const uint32_t* perm = sorted ? b->srt.perm : nullptr;
  if (sorted) {
    hipError_t e = gvk_sort_slots(&b->srt, b->n, b->kslot, b->kcount, st);
    if (e != hipSuccess) return e;
    e = gvk_unpack_perm(b->sig64, b->dig32, perm, b->n, C, b->in_r, b->in_s, b->in_e, st);
    if (e != hipSuccess) return e;
  } else if (b->unpacked != 1) {                 // 2: the key rows only (in-batch grouping)
    hipLaunchKernelGGL(gv::k_unpack, grd, blk, 0, st, b->unpacked ? (const uint8_t*)nullptr : b->pub33, b->sig64,
                       b->dig32, b->n, C, b->in_x, b->in_pfx, b->in_r, b->in_s, b->in_e);
  }
  if (b->msg_blob)
    hipLaunchKernelGGL(gv::k_sha256, grd, blk, 0, st, b->msg_blob, b->msg_off, b->msg_len, b->n, C,
                       b->in_e, perm);
  if (b->ev[0]) (void)hipEventRecord(b->ev[0], st);
  {
    const uint32_t M = b->inv_m ? b->inv_m : gvk_inv_m(C);
    const uint32_t waves = (C / 64 + M - 1) / M;
    // scratch for w and the prefix products: the digit rows.  k_prep reads
    // its lane's w before writing that lane's digits (same lane, same rows).
    uint32_t* w = b->digits;                   // rows 0..8
    uint32_t* pre = b->digits + (size_t)9 * C; // rows 9..17
    hipLaunchKernelGGL(gv::k_scalar_inv, dim3((waves + 3) / 4), blk, 0, st, C, b->in_s, w, pre, M);
    if (b->keys_ready) (void)hipStreamWaitEvent(st, b->keys_ready, 0);   // grouped keys built beside s^-1
    if (b->ev[1]) (void)hipEventRecord(b->ev[1], st);
    if (kg)
      hipLaunchKernelGGL((gv::k_prep<true, true, true, false, true>), grd, blk, 0, st, C, b->n, (const uint32_t*)nullptr,
                         (const uint32_t*)nullptr, b->in_r, b->in_s, b->in_e, (const uint32_t*)w, b->digits,
                         (uint32_t*)nullptr, (uint32_t*)nullptr, b->flags, sorted ? b->srt.kslot : b->kslot,
                         b->kok, b->kcount, b->in_pfx);
    else if (kw)
      hipLaunchKernelGGL((gv::k_prep<true, true, true, true>), grd, blk, 0, st, C, b->n, (const uint32_t*)nullptr,
                         (const uint32_t*)nullptr, b->in_r, b->in_s, b->in_e, (const uint32_t*)w, b->digits,
                         (uint32_t*)nullptr, (uint32_t*)nullptr, b->flags, sorted ? b->srt.kslot : b->kslot,
                         b->kok, b->kcount, b->in_pfx);
    else if (k6)
      hipLaunchKernelGGL((gv::k_prep<true, true, true>), grd, blk, 0, st, C, b->n, (const uint32_t*)nullptr,
                         (const uint32_t*)nullptr, b->in_r, b->in_s, b->in_e, (const uint32_t*)w, b->digits,
                         (uint32_t*)nullptr, (uint32_t*)nullptr, b->flags, sorted ? b->srt.kslot : b->kslot,
                         b->kok, b->kcount, b->in_pfx);
    else if (gf)
      hipLaunchKernelGGL((gv::k_prep<true, false, true>), grd, blk, 0, st, C, b->n, (const uint32_t*)nullptr,
                         (const uint32_t*)nullptr, b->in_r, b->in_s, b->in_e, (const uint32_t*)w, b->digits,
                         (uint32_t*)nullptr, (uint32_t*)nullptr, b->flags, sorted ? b->srt.kslot : b->kslot,
                         b->kok, b->kcount, b->in_pfx);
    else if (b->kslot)   // keyed: in_pfx doubles as the clamped-slot row for k_ecmult
      hipLaunchKernelGGL(gv::k_prep<true>, grd, blk, 0, st, C, b->n, (const uint32_t*)nullptr,
                         (const uint32_t*)nullptr, b->in_r, b->in_s, b->in_e, (const uint32_t*)w, b->digits,
                         (uint32_t*)nullptr, (uint32_t*)nullptr, b->flags, sorted ? b->srt.kslot : b->kslot,
                         b->kok, b->kcount, b->in_pfx);
    else if (gfp)
      hipLaunchKernelGGL((gv::k_prep<false, false, true>), grd, blk, 0, st, C, b->n, b->in_x, b->in_pfx, b->in_r,
                         b->in_s, b->in_e, (const uint32_t*)w, b->digits, b->qtab, b->zq, b->flags,
                         (const uint32_t*)nullptr, (const uint32_t*)nullptr, 0u, (uint32_t*)nullptr);
    else
      hipLaunchKernelGGL(gv::k_prep<false>, grd, blk, 0, st, C, b->n, b->in_x, b->in_pfx, b->in_r, b->in_s,
                         b->in_e, (const uint32_t*)w, b->digits, b->qtab, b->zq, b->flags,
                         (const uint32_t*)nullptr, (const uint32_t*)nullptr, 0u, (uint32_t*)nullptr);
  }
  if (b->ev[2]) (void)hipEventRecord(b->ev[2], st);
  hipStream_t se = st;
  if (b->st_ecm) {                             // the ladder on its own (high-priority) stream
    (void)hipEventRecord(b->ecm_ready, st);
    (void)hipStreamWaitEvent(b->st_ecm, b->ecm_ready, 0);
    se = b->st_ecm;
  }
  if (b->ev_ecm_start) (void)hipEventRecord(b->ev_ecm_start, se);
  if (b->bits_wait && !sorted) (void)hipStreamWaitEvent(se, b->bits_wait, 0);   // the ladder writes the bits
#define GV_KG_LAUNCH(NG)                                                                                      \
  hipLaunchKernelGGL((gv::k_ecmult_kn<GV_QW, NG>), grd, blk, 0, se, b->gtab6, b->n, C, b->digits, b->kqt, b->kqt2, \
                     b->kzq, b->flags, b->in_r, sorted ? b->srt.bits : b->bits, (const uint32_t*)b->in_pfx, b->kC)
  if (kg && b->k6 == 4)
    GV_KG_LAUNCH(4);
  else if (kg && b->k6 == 6)
    GV_KG_LAUNCH(6);
  else if (kg && b->k6 == 7)
    GV_KG_LAUNCH(7);
  else if (kg && b->k6 == 9)
    GV_KG_LAUNCH(9);
#undef GV_KG_LAUNCH
  else if (kg)
    return hipErrorInvalidValue;
  else if (kw && b->k6 == GV_KW_NG1)
    hipLaunchKernelGGL((gv::k_ecmult_kn<GV_KW_QW, GV_KW_NG1>), grd, blk, 0, se, b->gtab6, b->n, C, b->digits,
                       b->kqt, b->kqt2, b->kzq, b->flags, b->in_r, sorted ? b->srt.bits : b->bits,
                       (const uint32_t*)b->in_pfx, b->kC);
  else if (kw)
    hipLaunchKernelGGL((gv::k_ecmult_kn<GV_KW_QW, GV_KW_NG2>), grd, blk, 0, se, b->gtab6, b->n, C, b->digits,
                       b->kqt, b->kqt2, b->kzq, b->flags, b->in_r, sorted ? b->srt.bits : b->bits,
                       (const uint32_t*)b->in_pfx, b->kC);
  else if (k6 && b->k6 == GV_KN_ARENA_NG)
    hipLaunchKernelGGL((gv::k_ecmult_kn<GV_K6_QW, GV_KN_ARENA_NG>), grd, blk, 0, se, b->gtab6, b->n, C, b->digits, b->kqt, b->kqt2,
                       b->kzq, b->flags, b->in_r, sorted ? b->srt.bits : b->bits, (const uint32_t*)b->in_pfx, b->kC);
  else if (k6)
    hipLaunchKernelGGL((gv::k_ecmult_kn<GV_K6_QW, 4>), grd, blk, 0, se, b->gtab6, b->n, C, b->digits, b->kqt, b->kqt2, b->kzq,
                       b->flags, b->in_r, sorted ? b->srt.bits : b->bits, (const uint32_t*)b->in_pfx, b->kC);
  else if (gf)
    hipLaunchKernelGGL(gv::k_ecmult_k4<true>, grd, blk, 0, se, b->gtabf, b->gtab4, b->n, C, b->digits, b->kqt,
                       b->kqt2, b->kzq, b->flags, b->in_r, sorted ? b->srt.bits : b->bits,
                       (const uint32_t*)b->in_pfx, b->kC);
  else if (b->kslot && b->gtab4)
    hipLaunchKernelGGL(gv::k_ecmult_k4<false>, grd, blk, 0, se, b->gtab, b->gtab4, b->n, C, b->digits, b->kqt, b->kqt2,
                       b->kzq, b->flags, b->in_r, sorted ? b->srt.bits : b->bits, (const uint32_t*)b->in_pfx,
                       b->kC);
  else if (b->kslot)
    hipLaunchKernelGGL(gv::k_ecmult<true>, grd, blk, 0, se, b->gtab, b->n, C, b->digits, b->kqt, b->kzq,
                       b->flags, b->in_r, b->bits, (const uint32_t*)b->in_pfx, b->kC);
  else if (gfp)
    hipLaunchKernelGGL((gv::k_ecmult<false, true>), grd, blk, 0, se, b->gtabf, b->n, C, b->digits,
                       (const uint32_t*)b->qtab, (const uint32_t*)b->zq, b->flags, b->in_r, b->bits,
                       (const uint32_t*)nullptr, 0u);
  else
    hipLaunchKernelGGL(gv::k_ecmult<false>, grd, blk, 0, se, b->gtab, b->n, C, b->digits,
                       (const uint32_t*)b->qtab, (const uint32_t*)b->zq, b->flags, b->in_r, b->bits,
                       (const uint32_t*)nullptr, 0u);
  if (b->ev[3]) (void)hipEventRecord(b->ev[3], se);
  if (sorted) {
    if (b->bits_wait) (void)hipStreamWaitEvent(se, b->bits_wait, 0);
    const hipError_t e = gvk_unsort_bits(b->n, b->srt.pos, b->srt.bits, b->bits, se);
    if (b->bits_done) (void)hipEventRecord(b->bits_done, se);
    return e;
  }
  if (b->bits_done) (void)hipEventRecord(b->bits_done, se);
  return hipGetLastError();
}

hipError_t gvk_gen_glat(uint32_t* glat, hipStream_t st) {
  hipLaunchKernelGGL(gv::k_gen_glat, dim3(1), dim3(GV_LGRP * 2 * GV_QTAB_N), 0, st, glat);
  return hipGetLastError();
}

// The key-table launches (k_keys_chain, k_keys_fwd, k_keys_back) over n keys
// whose rows in_x / in_pfx (stride C) are unpacked.  Scratch (gv_kernels.h
// gvk_keys_scratch_words): ratio rows, the E rows, the forward entries.
}  // extern "C"
template <int QW, int NG>
static hipError_t keys_tables_launch(uint32_t n, uint32_t C, const uint32_t* in_x, const uint32_t* in_pfx,
                                     uint32_t* scratch, int with_qe, uint32_t base, uint32_t* kqt, uint32_t* kzq,
                                     uint32_t kC, uint32_t* kok, uint32_t* kqt2, uint32_t* kzq2, hipStream_t st) {
  if (n == 0) return hipSuccess;
  constexpr int NT = gv::KLayout<QW, NG>::NT;
  const uint32_t CL = gvk_keys_lanes(n, NG);
  uint32_t* qr = scratch;
  uint32_t* er = qr + (size_t)(NT - 2) * 9 * CL;
  uint32_t* qe = with_qe ? er + (size_t)9 * CL : nullptr;
  hipLaunchKernelGGL((gv::k_keys_chain<QW, NG>), dim3((n + 255) / 256), dim3(GV_CHAIN_SPLIT ? 512 : 256), 0, st, n, C,
                     in_x, in_pfx, base, kqt, kC, kok, kqt2, kzq2, kzq);
  if (NG == 4) {
    // four groups: one launch, the quad trades its Zs by lane shuffles (the
    // last entry stays in registers; the E rows are unused)
    hipLaunchKernelGGL((gv::k_keys_tables<QW>), dim3(CL / 256), dim3(256), 0, st, n, CL, base, kqt, kzq, kC, kqt2, kzq2,
                       qr, qe);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((gv::k_keys_fwd<QW, NG>), dim3(CL / 256), dim3(256), 0, st, n, CL, base, kqt, kC, kqt2,
                     (const uint32_t*)kzq2, qr, qe, er, (const uint32_t*)kzq);
  hipLaunchKernelGGL((gv::k_keys_back<QW, NG>), dim3(CL / 256), dim3(256), 0, st, n, CL, base, kqt, kzq, kC, kqt2,
                     kzq2, (const uint32_t*)qr, (const uint32_t*)qe, (const uint32_t*)er);
  return hipGetLastError();
}

extern "C" {
uint32_t gvk_keys_lanes(uint32_t n, int ng) { return ((uint32_t)ng * n + 255u) / 256u * 256u; }
size_t gvk_keys_scratch_words(uint32_t n, int ng, int nt, int with_qe) {
  return (size_t)gvk_keys_lanes(n, ng) * ((size_t)(nt - 2) * 9 + 9 + (with_qe ? (size_t)nt * 18 : 0));
}

hipError_t gvk_keys_build_rows6(uint32_t n, uint32_t C, const uint32_t* in_x, const uint32_t* in_pfx,
                                uint32_t* scratch, int with_qe, uint32_t* kqt, uint32_t* kzq, uint32_t kC,
                                uint32_t* kok, uint32_t* kqt2, uint32_t* kzq2, hipStream_t st) {
  return keys_tables_launch<GV_K6_QW, 4>(n, C, in_x, in_pfx, scratch, with_qe, 0u, kqt, kzq, kC, kok, kqt2, kzq2, st);
}

hipError_t gvk_keys_build_rows_kg(uint32_t n, uint32_t C, const uint32_t* in_x, const uint32_t* in_pfx,
                                  uint32_t* scratch, int with_qe, uint32_t* kqt, uint32_t* kzq, uint32_t kC,
                                  uint32_t* kok, uint32_t* kqt2, uint32_t* kzq2, int ng, hipStream_t st) {
  switch (ng) {
    case 4: return keys_tables_launch<GV_QW, 4>(n, C, in_x, in_pfx, scratch, with_qe, 0u, kqt, kzq, kC, kok, kqt2, kzq2, st);
    case 6: return keys_tables_launch<GV_QW, 6>(n, C, in_x, in_pfx, scratch, with_qe, 0u, kqt, kzq, kC, kok, kqt2, kzq2, st);
    case 7: return keys_tables_launch<GV_QW, 7>(n, C, in_x, in_pfx, scratch, with_qe, 0u, kqt, kzq, kC, kok, kqt2, kzq2, st);
    case 9: return keys_tables_launch<GV_QW, 9>(n, C, in_x, in_pfx, scratch, with_qe, 0u, kqt, kzq, kC, kok, kqt2, kzq2, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t gvk_keys_build_wide(const uint8_t* pub33, uint32_t n, uint32_t C, uint32_t* in_x, uint32_t* in_pfx,
                               uint32_t* in_r, uint32_t* in_s, uint32_t* in_e, uint32_t* scratch, int with_qe,
                               uint32_t base, uint32_t* kqtw, uint32_t* kzqw, uint32_t kC, uint32_t* kok,
                               uint32_t* kqtw2, uint32_t* kzqw2, int ng, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (ng != GV_KW_NG1 && ng != GV_KW_NG2) return hipErrorInvalidValue;
  const dim3 blk(256), grd(C / 256);
  hipLaunchKernelGGL(gv::k_unpack, grd, blk, 0, st, pub33, (const uint8_t*)nullptr, (const uint8_t*)nullptr, n, C,
                     in_x, in_pfx, in_r, in_s, in_e);
  if (ng == GV_KW_NG1)
    return keys_tables_launch<GV_KW_QW, GV_KW_NG1>(n, C, in_x, in_pfx, scratch, with_qe, base, kqtw, kzqw, kC, kok,
                                                   kqtw2, kzqw2, st);
  return keys_tables_launch<GV_KW_QW, GV_KW_NG2>(n, C, in_x, in_pfx, scratch, with_qe, base, kqtw, kzqw, kC, kok,
                                                 kqtw2, kzqw2, st);
}

hipError_t gvk_keys_build(const uint8_t* pub33, uint32_t n, uint32_t C, uint32_t* in_x, uint32_t* in_pfx,
                          uint32_t* in_r, uint32_t* in_s, uint32_t* in_e, uint32_t* scratch, int with_qe,
                          uint32_t base, uint32_t* kqt, uint32_t* kzq, uint32_t kC, uint32_t* kok, uint32_t* kqt2,
                          uint32_t* kzq2, hipStream_t st) {
  const dim3 blk(256), grd(C / 256);
  hipLaunchKernelGGL(gv::k_unpack, grd, blk, 0, st, pub33, (const uint8_t*)nullptr, (const uint8_t*)nullptr, n, C,
                     in_x, in_pfx, in_r, in_s, in_e);
  return keys_tables_launch<GV_QW, GV_LGRP>(n, C, in_x, in_pfx, scratch, with_qe, base, kqt, kzq, kC, kok, kqt2, kzq2,
                                            st);
}

hipError_t gvk_keys_build6(const uint8_t* pub33, uint32_t n, uint32_t C, uint32_t* in_x, uint32_t* in_pfx,
                           uint32_t* in_r, uint32_t* in_s, uint32_t* in_e, uint32_t* scratch, int with_qe,
                           uint32_t base, uint32_t* kqt6, uint32_t* kzq6, uint32_t kC, uint32_t* kok, uint32_t* kqt62,
                           uint32_t* kzq62, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const dim3 blk(256), grd(C / 256);
  hipLaunchKernelGGL(gv::k_unpack, grd, blk, 0, st, pub33, (const uint8_t*)nullptr, (const uint8_t*)nullptr, n, C,
                     in_x, in_pfx, in_r, in_s, in_e);
  return keys_tables_launch<GV_K6_QW, GV_KN_ARENA_NG>(n, C, in_x, in_pfx, scratch, with_qe, base, kqt6, kzq6, kC, kok,
                                                       kqt62, kzq62, st);
}

hipError_t gvk_keys_point(uint32_t n, const uint32_t* slots, const uint32_t* kqt, const uint32_t* kzq, uint32_t kC,
                          const uint32_t* kok, uint32_t kcount, uint8_t* out_xy, uint8_t* out_ok, hipStream_t st) {
  hipLaunchKernelGGL(gv::k_keys_point, dim3((n + 255) / 256), dim3(256), 0, st, n, slots, kqt, kzq, kC, kok, kcount,
                     out_xy, out_ok);
  return hipGetLastError();
}

hipError_t gvk_sha256(const uint8_t* blob, const uint64_t* off, const uint32_t* len, uint32_t n, uint32_t C,
                      uint32_t* e, hipStream_t st) {
  hipLaunchKernelGGL(gv::k_sha256, dim3(C / 256), dim3(256), 0, st, blob, off, len, n, C, e, (const uint32_t*)nullptr);
  return hipGetLastError();
}

hipError_t gvk_unpack(const uint8_t* pub33, const uint8_t* sig64, const uint8_t* dig32, uint32_t n, uint32_t C,
                      uint32_t* x, uint32_t* pfx, uint32_t* r, uint32_t* s, uint32_t* e, hipStream_t st) {
  hipLaunchKernelGGL(gv::k_unpack, dim3(C / 256), dim3(256), 0, st, pub33, sig64, dig32, n, C, x, pfx, r, s, e);
  return hipGetLastError();
}

hipError_t gvk_dedupe(uint32_t n, uint32_t C, const uint32_t* x, const uint32_t* pfx, uint32_t* table, uint32_t tslots,
                      uint32_t* rep, uint32_t* uid, uint32_t* count, uint32_t* kslot, uint32_t capU, uint32_t CU,
                      uint32_t* kx, uint32_t* kpfx, hipStream_t st) {
  const dim3 blk(256), grd((n + 255) / 256);
  if (hipMemsetAsync(table, 0xFF, (size_t)tslots * 4, st) != hipSuccess ||
      hipMemsetAsync(count, 0, 4, st) != hipSuccess)
    return hipErrorUnknown;
  hipLaunchKernelGGL(gv::k_dedupe, grd, blk, 0, st, n, C, x, pfx, table, tslots - 1, rep);
  hipLaunchKernelGGL(gv::k_dedupe_assign, grd, blk, 0, st, n, C, x, pfx, (const uint32_t*)rep, uid, count, capU, CU,
                     kx, kpfx);
  hipLaunchKernelGGL(gv::k_dedupe_map, grd, blk, 0, st, n, (const uint32_t*)rep, (const uint32_t*)uid, kslot);
  return hipGetLastError();
}

hipError_t gvk_keys_build_rows(uint32_t n, uint32_t C, const uint32_t* in_x, const uint32_t* in_pfx,
                               uint32_t* scratch, int with_qe, uint32_t* kqt, uint32_t* kzq, uint32_t kC,
                               uint32_t* kok, uint32_t* kqt2, uint32_t* kzq2, hipStream_t st) {
  return keys_tables_launch<GV_QW, GV_LGRP>(n, C, in_x, in_pfx, scratch, with_qe, 0u, kqt, kzq, kC, kok, kqt2, kzq2,
                                            st);
}

#if GV_STAMP
hipError_t gvk_stamps_read(uint64_t* host, size_t n_u64) {
  const size_t cap = (size_t)2 * GV_STAMP_WAVES * 6;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(gv::g_stamps), std::min(n_u64, cap) * 8, 0, hipMemcpyDeviceToHost);
}
#endif

hipError_t gvk_debug(int op, uint32_t n, const uint32_t* in, uint32_t* out, hipStream_t st) {
  hipLaunchKernelGGL(gv::k_debug, dim3((n + 255) / 256), dim3(256), 0, st, op, n, in, out);
  return hipGetLastError();
}

}  // extern "C"
