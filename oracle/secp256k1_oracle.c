/*
 * secp256k1_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's signature-verification semantics, used
 * exclusively as the parity checker by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  Nothing in the product path (libgpuverify)
 * links, loads or calls this file.
 *
 * What it restates (the reference's Go path is not compilable here -- no Go
 * toolchain, and the arithmetic lives in third-party modules absent from
 * /root/reference):
 *   - x/auth/ante/sigverify.go:210  pubKey.VerifyBytes(signBytes, sig)
 *   - tendermint v0.33.4 crypto/secp256k1/secp256k1_nocgo.go  VerifyBytes:
 *       len(sig)==64, btcec.ParsePubKey, S <= N/2 (low-S), Signature.Verify
 *       over crypto.Sha256(msg)                          -> oracle_verify_bytes
 *   - btcsuite/btcd v0.20.1-beta btcec/pubkey.go ParsePubKey + decompressPoint
 *       (prefix 0x02/0x03, y = c^((p+1)/4), y^2==c, parity, X<P, Y<P,
 *       IsOnCurve)                                       -> parse_pubkey
 *   - btcec/btcec.go ScalarBaseMult (byte-indexed precomputed table
 *       "bytePoints", restated as base_table), ScalarMult, Add (complete
 *       affine addition, (0,0) = point at infinity)     -> base_mult, point_mult, ge_add
 *   - go1.14 crypto/ecdsa.Verify/verifyGeneric/hashToInt: 0<r,s<N,
 *       w=s^-1, u1=e*w, u2=r*w, R=u1*G+u2*Q, R==(0,0) -> false,
 *       R.x mod N == r                                   -> oracle_verify_digest
 *   - btcec signRFC6979/nonceRFC6979 (RFC 6979 HMAC-SHA256 nonce, low-S
 *       normalisation) and tendermint GenPrivKeySecp256k1 -- used only to
 *       MAKE test/bench inputs                           -> oracle_sign, oracle_privkey_from_secret
 *
 * Parity pinning (see DESIGN.md "Oracle"): k*G + SEC1 compression is pinned by
 * the reference's crypto/hd/testdata/test.json known-answer vectors; ECDSA
 * accept/reject is cross-checked against OpenSSL 3 (independent implementation)
 * and the pure-Python restatement oracle/secp_ref.py.  The reference's own tests
 * hold no ECDSA accept/reject vectors.
 *
 * Representation: 4 x 64-bit little-endian limbs, unsigned __int128 products,
 * every field/scalar value kept canonical (fully reduced) -- clarity over speed.
 */
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } u256;

/* ------------------------------------------------------------------ SHA-256 */
static const uint32_t SHA_K[64] = {
  0x428a2f98,0x71374491,0xb5c0fbcf,0xe9b5dba5,0x3956c25b,0x59f111f1,0x923f82a4,0xab1c5ed5,
  0xd807aa98,0x12835b01,0x243185be,0x550c7dc3,0x72be5d74,0x80deb1fe,0x9bdc06a7,0xc19bf174,
  0xe49b69c1,0xefbe4786,0x0fc19dc6,0x240ca1cc,0x2de92c6f,0x4a7484aa,0x5cb0a9dc,0x76f988da,
  0x983e5152,0xa831c66d,0xb00327c8,0xbf597fc7,0xc6e00bf3,0xd5a79147,0x06ca6351,0x14292967,
  0x27b70a85,0x2e1b2138,0x4d2c6dfc,0x53380d13,0x650a7354,0x766a0abb,0x81c2c92e,0x92722c85,
  0xa2bfe8a1,0xa81a664b,0xc24b8b70,0xc76c51a3,0xd192e819,0xd6990624,0xf40e3585,0x106aa070,
  0x19a4c116,0x1e376c08,0x2748774c,0x34b0bcb5,0x391c0cb3,0x4ed8aa4a,0x5b9cca4f,0x682e6ff3,
  0x748f82ee,0x78a5636f,0x84c87814,0x8cc70208,0x90befffa,0xa4506ceb,0xbef9a3f7,0xc67178f2};

typedef struct { uint32_t h[8]; uint8_t buf[64]; uint64_t total; size_t fill; } sha256_ctx;

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha256_block(uint32_t h[8], const uint8_t* p) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = (uint32_t)p[4*i] << 24 | (uint32_t)p[4*i+1] << 16 | (uint32_t)p[4*i+2] << 8 | p[4*i+3];
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = ROR(w[i-15], 7) ^ ROR(w[i-15], 18) ^ (w[i-15] >> 3);
    uint32_t s1 = ROR(w[i-2], 17) ^ ROR(w[i-2], 19) ^ (w[i-2] >> 10);
    w[i] = w[i-16] + s0 + w[i-7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = hh + S1 + ch + SHA_K[i] + w[i];
    uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
static void sha256_init(sha256_ctx* c) {
  static const uint32_t iv[8] = {0x6a09e667,0xbb67ae85,0x3c6ef372,0xa54ff53a,0x510e527f,0x9b05688c,0x1f83d9ab,0x5be0cd19};
  memcpy(c->h, iv, sizeof iv); c->total = 0; c->fill = 0;
}
static void sha256_update(sha256_ctx* c, const uint8_t* p, size_t n) {
  c->total += n;
  while (n) {
    size_t take = 64 - c->fill; if (take > n) take = n;
    memcpy(c->buf + c->fill, p, take); c->fill += take; p += take; n -= take;
    if (c->fill == 64) { sha256_block(c->h, c->buf); c->fill = 0; }
  }
}
static void sha256_final(sha256_ctx* c, uint8_t out[32]) {
  uint64_t bits = c->total * 8;
  uint8_t pad = 0x80; sha256_update(c, &pad, 1);
  uint8_t z = 0; while (c->fill != 56) sha256_update(c, &z, 1);
  uint8_t len[8]; for (int i = 0; i < 8; ++i) len[i] = (uint8_t)(bits >> (56 - 8*i));
  sha256_update(c, len, 8);
  for (int i = 0; i < 8; ++i) { out[4*i] = c->h[i] >> 24; out[4*i+1] = c->h[i] >> 16; out[4*i+2] = c->h[i] >> 8; out[4*i+3] = c->h[i]; }
}
void oracle_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  sha256_ctx c; sha256_init(&c); sha256_update(&c, msg, len); sha256_final(&c, out);
}
static void hmac_sha256(const uint8_t* key, size_t klen, const uint8_t* m1, size_t l1,
                        const uint8_t* m2, size_t l2, const uint8_t* m3, size_t l3,
                        const uint8_t* m4, size_t l4, uint8_t out[32]) {
  uint8_t k[64] = {0}, ipad[64], opad[64], inner[32];
  if (klen > 64) oracle_sha256(key, klen, k); else memcpy(k, key, klen);
  for (int i = 0; i < 64; ++i) { ipad[i] = k[i] ^ 0x36; opad[i] = k[i] ^ 0x5c; }
  sha256_ctx c; sha256_init(&c); sha256_update(&c, ipad, 64);
  if (l1) sha256_update(&c, m1, l1);
  if (l2) sha256_update(&c, m2, l2);
  if (l3) sha256_update(&c, m3, l3);
  if (l4) sha256_update(&c, m4, l4);
  sha256_final(&c, inner);
  sha256_init(&c); sha256_update(&c, opad, 64); sha256_update(&c, inner, 32); sha256_final(&c, out);
}

/* --------------------------------------------------------- 256-bit helpers */
static void u256_from_be(u256* r, const uint8_t* b) {
  for (int i = 0; i < 4; ++i) {
    uint64_t w = 0; for (int j = 0; j < 8; ++j) w = (w << 8) | b[(3 - i) * 8 + j];
    r->v[i] = w;
  }
}
static void u256_to_be(uint8_t* b, const u256* a) {
  for (int i = 0; i < 4; ++i) for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (uint8_t)(a->v[i] >> (56 - 8 * j));
}
static int u256_cmp(const u256* a, const u256* b) {
  for (int i = 3; i >= 0; --i) { if (a->v[i] < b->v[i]) return -1; if (a->v[i] > b->v[i]) return 1; }
  return 0;
}
static int u256_is_zero(const u256* a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }
static uint64_t u256_add(u256* r, const u256* a, const u256* b) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) { c += (u128)a->v[i] + b->v[i]; r->v[i] = (uint64_t)c; c >>= 64; }
  return (uint64_t)c;
}
static uint64_t u256_sub(u256* r, const u256* a, const u256* b) {
  uint64_t borrow = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a->v[i] - b->v[i] - borrow;
    r->v[i] = (uint64_t)d; borrow = (uint64_t)(d >> 64) & 1;
  }
  return borrow;
}
static int u256_bit(const u256* a, int i) { return (int)((a->v[i >> 6] >> (i & 63)) & 1); }

/* ------------------------------------------------------------- constants */
static const u256 P  = {{0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL}};
static const u256 N  = {{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL}};
static const u256 HALF_N = {{0xDFE92F46681B20A0ULL, 0x5D576E7357A4501DULL, 0xFFFFFFFFFFFFFFFFULL, 0x7FFFFFFFFFFFFFFFULL}};
static const u256 GX = {{0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL, 0x79BE667EF9DCBBACULL}};
static const u256 GY = {{0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL, 0x483ADA7726A3C465ULL}};
/* 2^256 mod p and 2^256 mod n */
static const uint64_t P_FOLD = 0x1000003D1ULL;
static const u256 N_FOLD = {{0x402DA1732FC9BEBFULL, 0x4551231950B75FC4ULL, 0x1ULL, 0x0ULL}};

/* ------------------------------------------------------------ field mod p */
typedef u256 fe;
static void fe_reduce_once(fe* r) { fe t; if (!u256_sub(&t, r, &P)) *r = t; }
static void fe_mul(fe* r, const fe* a, const fe* b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) { c += (u128)a->v[i] * b->v[j] + t[i + j]; t[i + j] = (uint64_t)c; c >>= 64; }
    t[i + 4] = (uint64_t)c;
  }
  /* t = L + H*2^256 == L + H*P_FOLD (mod p) */
  u128 c = 0; uint64_t m[5];
  for (int i = 0; i < 4; ++i) { c += (u128)t[4 + i] * P_FOLD + t[i]; m[i] = (uint64_t)c; c >>= 64; }
  m[4] = (uint64_t)c;
  c = (u128)m[4] * P_FOLD;
  for (int i = 0; i < 4; ++i) { c += m[i]; r->v[i] = (uint64_t)c; c >>= 64; }
  if (c) { /* one more wrap: value < 2^256 + small, add P_FOLD again */
    c = P_FOLD;
    for (int i = 0; i < 4; ++i) { c += r->v[i]; r->v[i] = (uint64_t)c; c >>= 64; }
  }
  fe_reduce_once(r);
}
static void fe_sqr(fe* r, const fe* a) { fe_mul(r, a, a); }
static void fe_add(fe* r, const fe* a, const fe* b) {
  uint64_t c = u256_add(r, a, b);
  if (c) { fe t; u256 pf = {{P_FOLD, 0, 0, 0}}; u256_add(&t, r, &pf); *r = t; }
  fe_reduce_once(r);
}
static void fe_sub(fe* r, const fe* a, const fe* b) {
  if (u256_sub(r, a, b)) u256_add(r, r, &P);
}
static void fe_neg(fe* r, const fe* a) { fe z = {{0, 0, 0, 0}}; fe_sub(r, &z, a); }
static void fe_pow(fe* r, const fe* a, const u256* e) {
  fe acc = {{1, 0, 0, 0}};
  for (int i = 255; i >= 0; --i) { fe_sqr(&acc, &acc); if (u256_bit(e, i)) fe_mul(&acc, &acc, a); }
  *r = acc;
}
static void fe_inv(fe* r, const fe* a) {
  u256 e = P; e.v[0] -= 2; fe_pow(r, a, &e);
}
static int fe_eq(const fe* a, const fe* b) { return u256_cmp(a, b) == 0; }

/* ----------------------------------------------------------- scalar mod n */
typedef u256 sc;
static void sc_reduce_once(sc* r) { sc t; if (!u256_sub(&t, r, &N)) *r = t; }
/* reduce a 512-bit value (8 limbs) mod n by folding 2^256 == N_FOLD (129 bits) */
static void sc_reduce512(sc* r, const uint64_t t_in[8]) {
  uint64_t t[8]; memcpy(t, t_in, sizeof t);
  for (;;) {
    int hi_zero = (t[4] | t[5] | t[6] | t[7]) == 0;
    if (hi_zero) break;
    uint64_t m[8] = {0};
    /* m = H * N_FOLD  (H: 4 limbs, N_FOLD: 3 limbs) */
    for (int i = 0; i < 4; ++i) {
      u128 c = 0;
      for (int j = 0; j < 3; ++j) { c += (u128)t[4 + i] * N_FOLD.v[j] + m[i + j]; m[i + j] = (uint64_t)c; c >>= 64; }
      int k = i + 3; while (c && k < 8) { c += m[k]; m[k] = (uint64_t)c; c >>= 64; ++k; }
    }
    /* t = L + m */
    u128 c = 0;
    for (int i = 0; i < 8; ++i) { c += (u128)m[i] + (i < 4 ? t[i] : 0); t[i] = (uint64_t)c; c >>= 64; }
  }
  u256 x = {{t[0], t[1], t[2], t[3]}};
  sc_reduce_once(&x); sc_reduce_once(&x);
  *r = x;
}
static void sc_mul(sc* r, const sc* a, const sc* b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) { c += (u128)a->v[i] * b->v[j] + t[i + j]; t[i + j] = (uint64_t)c; c >>= 64; }
    t[i + 4] = (uint64_t)c;
  }
  sc_reduce512(r, t);
}
static void sc_inv(sc* r, const sc* a) {
  u256 e = N; e.v[0] -= 2;
  sc acc = {{1, 0, 0, 0}};
  for (int i = 255; i >= 0; --i) { sc_mul(&acc, &acc, &acc); if (u256_bit(&e, i)) sc_mul(&acc, &acc, a); }
  *r = acc;
}
static void sc_add(sc* r, const sc* a, const sc* b) {
  uint64_t c = u256_add(r, a, b);
  if (c) { u256_add(r, r, &N_FOLD); }
  sc_reduce_once(r);
}

/* --------------------------------------------------------------- group law */
/* Affine point; inf=1 encodes btcec's (0,0) point at infinity. */
typedef struct { fe x, y; int inf; } ge;
/* Jacobian point: (X/Z^2, Y/Z^3); inf flag instead of Z==0 tests */
typedef struct { fe x, y, z; int inf; } gej;

static void gej_set_ge(gej* r, const ge* a) {
  r->x = a->x; r->y = a->y; memset(&r->z, 0, sizeof r->z); r->z.v[0] = 1; r->inf = a->inf;
}
static void gej_double(gej* r, const gej* a) {
  if (a->inf) { *r = *a; return; }
  /* y == 0 cannot happen on secp256k1 (prime order, no 2-torsion) */
  fe A, B, C, D, E, F, t, x3, y3, z3;
  fe_sqr(&A, &a->x); fe_sqr(&B, &a->y); fe_sqr(&C, &B);
  fe_add(&t, &a->x, &B); fe_sqr(&t, &t); fe_sub(&t, &t, &A); fe_sub(&t, &t, &C); fe_add(&D, &t, &t);
  fe_add(&E, &A, &A); fe_add(&E, &E, &A);
  fe_sqr(&F, &E);
  fe_add(&t, &D, &D); fe_sub(&x3, &F, &t);
  fe_sub(&t, &D, &x3); fe_mul(&y3, &E, &t);
  fe_add(&C, &C, &C); fe_add(&C, &C, &C); fe_add(&C, &C, &C); fe_sub(&y3, &y3, &C);
  fe_mul(&z3, &a->y, &a->z); fe_add(&z3, &z3, &z3);
  r->x = x3; r->y = y3; r->z = z3; r->inf = 0;
}
/* complete addition r = a + b (Jacobian + Jacobian) */
static void gej_add(gej* r, const gej* a, const gej* b) {
  if (a->inf) { *r = *b; return; }
  if (b->inf) { *r = *a; return; }
  fe z1z1, z2z2, u1, u2, s1, s2, h, rr, t;
  fe_sqr(&z1z1, &a->z); fe_sqr(&z2z2, &b->z);
  fe_mul(&u1, &a->x, &z2z2); fe_mul(&u2, &b->x, &z1z1);
  fe_mul(&t, &b->z, &z2z2); fe_mul(&s1, &a->y, &t);
  fe_mul(&t, &a->z, &z1z1); fe_mul(&s2, &b->y, &t);
  fe_sub(&h, &u2, &u1); fe_sub(&rr, &s2, &s1);
  fe zero = {{0, 0, 0, 0}};
  if (fe_eq(&h, &zero)) {
    if (fe_eq(&rr, &zero)) { gej_double(r, a); return; }   /* P == Q */
    r->inf = 1; memset(&r->x, 0, sizeof(fe) * 3); return;  /* P == -Q */
  }
  fe hh, hhh, v, x3, y3, z3;
  fe_sqr(&hh, &h); fe_mul(&hhh, &h, &hh); fe_mul(&v, &u1, &hh);
  fe_sqr(&x3, &rr); fe_sub(&x3, &x3, &hhh); fe_sub(&x3, &x3, &v); fe_sub(&x3, &x3, &v);
  fe_sub(&t, &v, &x3); fe_mul(&y3, &rr, &t); fe_mul(&t, &s1, &hhh); fe_sub(&y3, &y3, &t);
  fe_mul(&z3, &a->z, &b->z); fe_mul(&z3, &z3, &h);
  r->x = x3; r->y = y3; r->z = z3; r->inf = 0;
}
static void ge_set_gej(ge* r, const gej* a) {
  if (a->inf) { memset(r, 0, sizeof *r); r->inf = 1; return; }
  fe zi, zi2, zi3; fe_inv(&zi, &a->z); fe_sqr(&zi2, &zi); fe_mul(&zi3, &zi2, &zi);
  fe_mul(&r->x, &a->x, &zi2); fe_mul(&r->y, &a->y, &zi3); r->inf = 0;
}
/* btcec Add(x1,y1,x2,y2): affine complete addition */
static void ge_add(ge* r, const ge* a, const ge* b) {
  gej ja, jb, jr; gej_set_ge(&ja, a); gej_set_ge(&jb, b); gej_add(&jr, &ja, &jb); ge_set_gej(r, &jr);
}

/* btcec ScalarMult(Bx, By, k): here a plain 4-bit fixed window, MSB first. */
static void point_mult(ge* r, const ge* q, const sc* k) {
  gej tab[16]; gej_set_ge(&tab[1], q); tab[0].inf = 1;
  for (int i = 2; i < 16; ++i) gej_add(&tab[i], &tab[i - 1], &tab[1]);
  gej acc; acc.inf = 1;
  for (int w = 63; w >= 0; --w) {
    for (int d = 0; d < 4; ++d) gej_double(&acc, &acc);
    int nib = (int)((k->v[w >> 4] >> ((w & 15) * 4)) & 15);
    if (nib) gej_add(&acc, &acc, &tab[nib]);
  }
  ge_set_gej(r, &acc);
}

/* btcec ScalarBaseMult: sum over the 32 bytes of k of bytePoints[i][byte]. */
static ge* base_table; /* [32][256] affine, table[i][b] = b * 2^(8i) * G */
static pthread_once_t base_once = PTHREAD_ONCE_INIT;
static void base_table_init(void) {
  base_table = (ge*)malloc(sizeof(ge) * 32 * 256);
  gej* jt = (gej*)malloc(sizeof(gej) * 32 * 256);
  gej base; base.x = GX; base.y = GY; memset(&base.z, 0, sizeof base.z); base.z.v[0] = 1; base.inf = 0;
  for (int i = 0; i < 32; ++i) {
    jt[i * 256].inf = 1;
    jt[i * 256 + 1] = base;
    for (int b = 2; b < 256; ++b) gej_add(&jt[i * 256 + b], &jt[i * 256 + b - 1], &base);
    for (int d = 0; d < 8; ++d) gej_double(&base, &base);
  }
  /* batch inversion of all Z (Montgomery trick) */
  int n = 32 * 256;
  fe* pre = (fe*)malloc(sizeof(fe) * n);
  fe acc = {{1, 0, 0, 0}};
  for (int i = 0; i < n; ++i) { pre[i] = acc; if (!jt[i].inf) fe_mul(&acc, &acc, &jt[i].z); }
  fe inv; fe_inv(&inv, &acc);
  for (int i = n - 1; i >= 0; --i) {
    if (jt[i].inf) { memset(&base_table[i], 0, sizeof(ge)); base_table[i].inf = 1; continue; }
    fe zi, zi2, zi3; fe_mul(&zi, &inv, &pre[i]); fe_mul(&inv, &inv, &jt[i].z);
    fe_sqr(&zi2, &zi); fe_mul(&zi3, &zi2, &zi);
    fe_mul(&base_table[i].x, &jt[i].x, &zi2); fe_mul(&base_table[i].y, &jt[i].y, &zi3); base_table[i].inf = 0;
  }
  free(pre); free(jt);
}
static void base_mult(ge* r, const sc* k) {
  pthread_once(&base_once, base_table_init);
  gej acc; acc.inf = 1;
  for (int i = 0; i < 32; ++i) {
    int byte = (int)((k->v[i >> 3] >> ((i & 7) * 8)) & 0xFF);
    if (!byte) continue;
    gej t; gej_set_ge(&t, &base_table[i * 256 + byte]); gej_add(&acc, &acc, &t);
  }
  ge_set_gej(r, &acc);
}

/* btcec ParsePubKey for a 33-byte compressed key (btcec/pubkey.go). */
static int parse_pubkey(ge* out, const uint8_t pub[33]) {
  uint8_t format = pub[0];
  int ybit = (format & 1) == 1;
  format &= (uint8_t)~1;
  if (format != 0x02) return 0;
  u256 x; u256_from_be(&x, pub + 1);
  /* decompressPoint: x3 = (x^3 + 7) mod p (big.Int arithmetic => uses x mod p) */
  fe xr = x; fe_reduce_once(&xr);
  fe x3, seven = {{7, 0, 0, 0}};
  fe_sqr(&x3, &xr); fe_mul(&x3, &x3, &xr); fe_add(&x3, &x3, &seven);
  u256 qp1d4 = {{0xFFFFFFFFBFFFFF0CULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0x3FFFFFFFFFFFFFFFULL}};
  fe y; fe_pow(&y, &x3, &qp1d4);
  if (ybit != (int)(y.v[0] & 1)) { u256 t; u256_sub(&t, &P, &y); y = t; }   /* y = P - y (big.Int) */
  fe y2; fe yr = y; fe_reduce_once(&yr); fe_sqr(&y2, &yr);
  if (!fe_eq(&y2, &x3)) return 0;                        /* "invalid square root" */
  if (ybit != (int)(y.v[0] & 1)) return 0;               /* "ybit doesn't match oddness" */
  if (u256_cmp(&x, &P) >= 0) return 0;                   /* "pubkey X parameter is >= to P" */
  if (u256_cmp(&y, &P) >= 0) return 0;                   /* "pubkey Y parameter is >= to P" */
  /* IsOnCurve: y^2 == x^3 + 7 */
  fe lhs, rhs; fe_sqr(&lhs, &y); fe_sqr(&rhs, &x); fe_mul(&rhs, &rhs, &x); fe_add(&rhs, &rhs, &seven);
  if (!fe_eq(&lhs, &rhs)) return 0;
  out->x = x; out->y = y; out->inf = 0;
  return 1;
}

/* ------------------------------------------------------------ public API */
int oracle_parse_pubkey(const uint8_t pub[33], uint8_t x_out[32], uint8_t y_out[32]) {
  ge q; if (!parse_pubkey(&q, pub)) return 0;
  if (x_out) u256_to_be(x_out, &q.x);
  if (y_out) u256_to_be(y_out, &q.y);
  return 1;
}

/* tendermint VerifyBytes with the message already hashed: digest = SHA256(msg). */
int oracle_verify_digest(const uint8_t pub[33], const uint8_t sig[64], const uint8_t digest[32]) {
  ge q;
  if (!parse_pubkey(&q, pub)) return 0;                  /* btcec.ParsePubKey error -> false */
  u256 r, s; u256_from_be(&r, sig); u256_from_be(&s, sig + 32);
  if (u256_cmp(&s, &HALF_N) > 0) return 0;               /* tendermint: reject high-S */
  /* crypto/ecdsa.Verify */
  if (u256_is_zero(&r) || u256_is_zero(&s)) return 0;
  if (u256_cmp(&r, &N) >= 0 || u256_cmp(&s, &N) >= 0) return 0;
  u256 e; u256_from_be(&e, digest);                      /* hashToInt: 32 bytes, no shift */
  sc_reduce_once(&e);
  sc w, u1, u2; sc_inv(&w, &s); sc_mul(&u1, &e, &w); sc_mul(&u2, &r, &w);
  ge p1, p2, R;
  base_mult(&p1, &u1);                                   /* ScalarBaseMult(u1.Bytes()) */
  point_mult(&p2, &q, &u2);                              /* ScalarMult(pub, u2.Bytes()) */
  ge_add(&R, &p1, &p2);                                  /* Add(x1,y1,x2,y2) */
  if (R.inf) return 0;                                   /* x==0 && y==0 -> false */
  u256 xr = R.x; sc_reduce_once(&xr);                    /* x.Mod(x, N) */
  return u256_cmp(&xr, &r) == 0;
}

int oracle_verify_bytes(const uint8_t pub[33], const uint8_t* msg, size_t msg_len,
                        const uint8_t* sig, size_t sig_len) {
  if (sig_len != 64) return 0;
  uint8_t d[32]; oracle_sha256(msg, msg_len, d);
  return oracle_verify_digest(pub, sig, d);
}

/* priv (32 BE) -> compressed pubkey (33). returns 0 if priv not in [1,n-1]. */
int oracle_pubkey(const uint8_t priv[32], uint8_t pub[33]) {
  u256 d; u256_from_be(&d, priv);
  if (u256_is_zero(&d) || u256_cmp(&d, &N) >= 0) return 0;
  ge q; base_mult(&q, &d);
  pub[0] = (uint8_t)(0x02 | (q.y.v[0] & 1)); u256_to_be(pub + 1, &q.x);
  return 1;
}

/* tendermint GenPrivKeySecp256k1(secret): (SHA256(secret) mod (n-1)) + 1 */
void oracle_privkey_from_secret(const uint8_t* secret, size_t len, uint8_t priv[32]) {
  uint8_t h[32]; oracle_sha256(secret, len, h);
  u256 fe_, nm1 = N; nm1.v[0] -= 1; u256_from_be(&fe_, h);
  if (u256_cmp(&fe_, &nm1) >= 0) u256_sub(&fe_, &fe_, &nm1);
  u256 one = {{1, 0, 0, 0}}; u256_add(&fe_, &fe_, &one);
  u256_to_be(priv, &fe_);
}

/* btcec signRFC6979: RFC 6979 nonce (HMAC-SHA256), r = (kG).x mod n,
 * s = k^-1 (e + d r) mod n, low-S normalised; output R||S (64 bytes). */
int oracle_sign(const uint8_t priv[32], const uint8_t digest[32], uint8_t sig[64]) {
  u256 d; u256_from_be(&d, priv);
  if (u256_is_zero(&d) || u256_cmp(&d, &N) >= 0) return 0;
  u256 z; u256_from_be(&z, digest); sc_reduce_once(&z);
  uint8_t x_oct[32], h_oct[32]; u256_to_be(x_oct, &d); u256_to_be(h_oct, &z);
  uint8_t V[32], K[32], T[32]; memset(V, 1, 32); memset(K, 0, 32);
  uint8_t b0 = 0, b1 = 1;
  hmac_sha256(K, 32, V, 32, &b0, 1, x_oct, 32, h_oct, 32, K);
  hmac_sha256(K, 32, V, 32, 0, 0, 0, 0, 0, 0, V);
  hmac_sha256(K, 32, V, 32, &b1, 1, x_oct, 32, h_oct, 32, K);
  hmac_sha256(K, 32, V, 32, 0, 0, 0, 0, 0, 0, V);
  for (;;) {
    hmac_sha256(K, 32, V, 32, 0, 0, 0, 0, 0, 0, V); memcpy(T, V, 32);
    u256 k; u256_from_be(&k, T);
    if (!u256_is_zero(&k) && u256_cmp(&k, &N) < 0) {
      ge R; base_mult(&R, &k);
      u256 r = R.x; sc_reduce_once(&r);
      if (!u256_is_zero(&r)) {
        u256 e; u256_from_be(&e, digest); sc_reduce_once(&e);
        sc kinv, s, t; sc_inv(&kinv, &k); sc_mul(&t, &d, &r); sc_add(&t, &t, &e); sc_mul(&s, &t, &kinv);
        if (u256_cmp(&s, &HALF_N) > 0) u256_sub(&s, &N, &s);
        if (!u256_is_zero(&s)) { u256_to_be(sig, &r); u256_to_be(sig + 32, &s); return 1; }
      }
    }
    hmac_sha256(K, 32, V, 32, &b0, 1, 0, 0, 0, 0, K);
    hmac_sha256(K, 32, V, 32, 0, 0, 0, 0, 0, 0, V);
  }
}

/* k*G and k*Q as affine 64-byte x||y (BE); inf -> returns 0 (used by KAT tests). */
int oracle_point_mul(const uint8_t pub[33], const uint8_t k32[32], uint8_t xy[64]) {
  u256 k; u256_from_be(&k, k32); ge r;
  if (pub == NULL) base_mult(&r, &k);
  else { ge q; if (!parse_pubkey(&q, pub)) return -1; point_mult(&r, &q, &k); }
  if (r.inf) return 0;
  u256_to_be(xy, &r.x); u256_to_be(xy + 32, &r.y); return 1;
}

/* ----------------------------------------------------- threaded batch API */
typedef struct {
  int kind; size_t lo, hi;
  const uint8_t *pub, *sig, *dig, *blob; const uint64_t* off; const uint32_t* len;
  const uint8_t* priv; uint8_t* out;
} job_t;
static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  for (size_t i = j->lo; i < j->hi; ++i) {
    switch (j->kind) {
      case 0: j->out[i] = (uint8_t)oracle_verify_digest(j->pub + 33 * i, j->sig + 64 * i, j->dig + 32 * i); break;
      case 1: j->out[i] = (uint8_t)oracle_verify_bytes(j->pub + 33 * i, j->blob + j->off[i], j->len[i], j->sig + 64 * i, 64); break;
      case 2: oracle_sign(j->priv + 32 * i, j->dig + 32 * i, j->out + 64 * i); break;
      case 3: oracle_pubkey(j->priv + 32 * i, j->out + 33 * i); break;
    }
  }
  return NULL;
}
static void run_jobs(job_t proto, size_t n, int threads) {
  pthread_once(&base_once, base_table_init);
  if (threads < 1) threads = 1;
  if ((size_t)threads > n) threads = n ? (int)n : 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  job_t* js = (job_t*)malloc(sizeof(job_t) * threads);
  for (int t = 0; t < threads; ++t) {
    js[t] = proto; js[t].lo = n * t / threads; js[t].hi = n * (t + 1) / threads;
    pthread_create(&th[t], NULL, worker, &js[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th); free(js);
}
void oracle_verify_digests(size_t n, const uint8_t* pub33, const uint8_t* sig64, const uint8_t* dig32,
                           uint8_t* out_ok, int threads) {
  job_t j = {0}; j.kind = 0; j.pub = pub33; j.sig = sig64; j.dig = dig32; j.out = out_ok;
  run_jobs(j, n, threads);
}
void oracle_verify_msgs(size_t n, const uint8_t* pub33, const uint8_t* sig64, const uint8_t* blob,
                        const uint64_t* off, const uint32_t* len, uint8_t* out_ok, int threads) {
  job_t j = {0}; j.kind = 1; j.pub = pub33; j.sig = sig64; j.blob = blob; j.off = off; j.len = len; j.out = out_ok;
  run_jobs(j, n, threads);
}
void oracle_sign_batch(size_t n, const uint8_t* priv32, const uint8_t* dig32, uint8_t* sig64, int threads) {
  job_t j = {0}; j.kind = 2; j.priv = priv32; j.dig = dig32; j.out = sig64;
  run_jobs(j, n, threads);
}
void oracle_pubkey_batch(size_t n, const uint8_t* priv32, uint8_t* pub33, int threads) {
  job_t j = {0}; j.kind = 3; j.priv = priv32; j.out = pub33;
  run_jobs(j, n, threads);
}
