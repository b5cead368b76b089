/*
 * gv_workload.c -- synthetic signed-transaction workload generator for
 * bench.py.  NOT the oracle: signatures are made
 * with OpenSSL 3 libcrypto (ECDSA_do_sign on NID_secp256k1, then tendermint's
 * low-S normalisation), keys follow tendermint GenPrivKeySecp256k1
 * ((SHA256(secret) mod (n-1)) + 1).  Expected verdicts are known by
 * construction: untouched items are valid, mutated (adversarial) items are
 * invalid.
 *
 * C1 sign bytes: StdSignBytes of a simapp bank MsgSend
 * (x/auth/types/stdtx.go:292-312, x/bank/types/msgs.go:43-45) with
 * from = addr_i, to = addr_{i+1}, amount 10foocoin, fee 0stake / gas 1000000,
 * memo "", chain-id "gv-bench", account number i, sequence 0.
 */
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/obj_mac.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

static const char* N_HEX = "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141";

/* ----------------------------------------------------------- RIPEMD-160 */
static uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static const int RL[80] = {0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,7,4,13,1,10,6,15,3,12,0,9,5,2,14,11,8,
  3,10,14,4,9,15,8,1,2,7,0,6,13,11,5,12,1,9,11,10,0,8,12,4,13,3,7,15,14,5,6,2,4,0,5,9,7,12,2,10,14,1,3,8,11,6,15,13};
static const int RR[80] = {5,14,7,0,9,2,11,4,13,6,15,8,1,10,3,12,6,11,3,7,0,13,5,10,14,15,8,12,4,9,1,2,
  15,5,1,3,7,14,6,9,11,8,12,2,10,0,4,13,8,6,4,1,3,11,15,0,5,12,2,13,9,7,10,14,12,15,10,4,1,5,8,7,6,2,13,14,0,3,9,11};
static const int SL[80] = {11,14,15,12,5,8,7,9,11,13,14,15,6,7,9,8,7,6,8,13,11,9,7,15,7,12,15,9,11,7,13,12,
  11,13,6,7,14,9,13,15,14,8,13,6,5,12,7,5,11,12,14,15,14,15,9,8,9,14,5,6,8,6,5,12,9,15,5,11,6,8,13,12,5,12,13,14,11,8,5,6};
static const int SR[80] = {8,9,9,11,13,15,15,5,7,7,8,11,14,14,12,6,9,13,15,7,12,8,9,11,7,7,12,7,6,15,13,11,
  9,7,15,11,8,6,6,14,12,13,5,14,13,13,7,5,15,5,8,11,14,14,6,14,6,9,12,9,12,5,15,8,8,5,12,9,12,5,14,6,8,13,6,5,15,13,11,11};
static uint32_t rf(int j, uint32_t x, uint32_t y, uint32_t z) {
  switch (j) { case 0: return x ^ y ^ z; case 1: return (x & y) | (~x & z); case 2: return (x | ~y) ^ z;
               case 3: return (x & z) | (y & ~z); default: return x ^ (y | ~z); }
}
static void ripemd160_32(const uint8_t in[32], uint8_t out[20]) {
  static const uint32_t KL[5] = {0, 0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xA953FD4E};
  static const uint32_t KR[5] = {0x50A28BE6, 0x5C4DD124, 0x6D703EF3, 0x7A6D76E9, 0};
  uint8_t blk[64] = {0}; memcpy(blk, in, 32); blk[32] = 0x80; blk[56] = 0x00; blk[57] = 0x01; /* 256 bits LE */
  uint32_t X[16]; for (int i = 0; i < 16; ++i) X[i] = blk[4*i] | blk[4*i+1] << 8 | blk[4*i+2] << 16 | (uint32_t)blk[4*i+3] << 24;
  uint32_t h[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
  uint32_t al = h[0], bl = h[1], cl = h[2], dl = h[3], el = h[4], ar = al, br = bl, cr = cl, dr = dl, er = el;
  for (int i = 0; i < 80; ++i) {
    int j = i / 16;
    uint32_t t = rol(al + rf(j, bl, cl, dl) + X[RL[i]] + KL[j], SL[i]) + el;
    al = el; el = dl; dl = rol(cl, 10); cl = bl; bl = t;
    t = rol(ar + rf(4 - j, br, cr, dr) + X[RR[i]] + KR[j], SR[i]) + er;
    ar = er; er = dr; dr = rol(cr, 10); cr = br; br = t;
  }
  uint32_t t = h[1] + cl + dr; h[1] = h[2] + dl + er; h[2] = h[3] + el + ar; h[3] = h[4] + al + br; h[4] = h[0] + bl + cr; h[0] = t;
  for (int i = 0; i < 5; ++i) for (int k = 0; k < 4; ++k) out[4*i+k] = (uint8_t)(h[i] >> (8*k));
}

/* ----------------------------------------------------------------- bech32 */
static uint32_t polymod(const uint8_t* v, size_t n) {
  static const uint32_t GEN[5] = {0x3b6a57b2, 0x26508e6d, 0x1ea119fa, 0x3d4233dd, 0x2a1462b3};
  uint32_t chk = 1;
  for (size_t i = 0; i < n; ++i) {
    uint32_t b = chk >> 25; chk = ((chk & 0x1ffffff) << 5) ^ v[i];
    for (int k = 0; k < 5; ++k) if ((b >> k) & 1) chk ^= GEN[k];
  }
  return chk;
}
static int bech32_cosmos(const uint8_t addr[20], char* out) {
  static const char* CS = "qpzry9x8gf2tvdw0s3jn54khce6mua7l";
  uint8_t v[64]; size_t nv = 0;
  const char* hrp = "cosmos";
  for (const char* p = hrp; *p; ++p) v[nv++] = (uint8_t)(*p >> 5);
  v[nv++] = 0;
  for (const char* p = hrp; *p; ++p) v[nv++] = (uint8_t)(*p & 31);
  size_t d0 = nv; uint32_t acc = 0; int bits = 0;
  for (int i = 0; i < 20; ++i) { acc = (acc << 8) | addr[i]; bits += 8; while (bits >= 5) { bits -= 5; v[nv++] = (acc >> bits) & 31; } }
  if (bits) v[nv++] = (acc << (5 - bits)) & 31;
  size_t dlen = nv - d0;
  for (int i = 0; i < 6; ++i) v[nv + i] = 0;
  uint32_t pm = polymod(v, nv + 6) ^ 1;
  int o = sprintf(out, "%s1", hrp);
  for (size_t i = 0; i < dlen; ++i) out[o++] = CS[v[d0 + i]];
  for (int i = 0; i < 6; ++i) out[o++] = CS[(pm >> (5 * (5 - i))) & 31];
  out[o] = 0;
  return o;
}

/* ------------------------------------------------------------------ keys */
typedef struct { size_t lo, hi; uint64_t seed; uint8_t *priv, *pub; } keyjob;
static void* key_worker(void* a) {
  keyjob* j = (keyjob*)a;
  EC_GROUP* grp = EC_GROUP_new_by_curve_name(NID_secp256k1);
  BN_CTX* ctx = BN_CTX_new();
  EC_GROUP_precompute_mult(grp, ctx);
  BIGNUM *n = NULL, *nm1 = BN_new(), *fe = BN_new();
  BN_hex2bn(&n, N_HEX); BN_copy(nm1, n); BN_sub_word(nm1, 1);
  EC_POINT* pt = EC_POINT_new(grp);
  for (size_t i = j->lo; i < j->hi; ++i) {
    uint8_t secret[22]; memcpy(secret, "gv-c2-", 6);
    for (int k = 0; k < 8; ++k) { secret[6 + k] = (uint8_t)(j->seed >> (8 * k)); secret[14 + k] = (uint8_t)((uint64_t)i >> (8 * k)); }
    uint8_t h[32]; SHA256(secret, sizeof secret, h);
    BN_bin2bn(h, 32, fe); BN_mod(fe, fe, nm1, ctx); BN_add_word(fe, 1);
    BN_bn2binpad(fe, j->priv + 32 * i, 32);
    EC_POINT_mul(grp, pt, fe, NULL, NULL, ctx);
    EC_POINT_point2oct(grp, pt, POINT_CONVERSION_COMPRESSED, j->pub + 33 * i, 33, ctx);
  }
  EC_POINT_free(pt); BN_free(n); BN_free(nm1); BN_free(fe); BN_CTX_free(ctx); EC_GROUP_free(grp);
  return NULL;
}

/* Derive nkeys (priv32, pub33) pairs. */
int gvw_keys(size_t nkeys, uint64_t seed, uint8_t* priv32, uint8_t* pub33, int threads) {
  if (threads < 1) threads = 1;
  pthread_t th[256]; keyjob js[256]; if (threads > 256) threads = 256;
  for (int t = 0; t < threads; ++t) {
    js[t].lo = nkeys * t / threads; js[t].hi = nkeys * (t + 1) / threads; js[t].seed = seed; js[t].priv = priv32; js[t].pub = pub33;
    pthread_create(&th[t], NULL, key_worker, &js[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  return 0;
}

/* ------------------------------------------------------- sign + mutate */
typedef struct {
  size_t lo, hi, nkeys; uint64_t seed; double adv;
  const uint8_t *priv, *pub; const uint32_t* kidx; const uint8_t* msgdig;
  uint8_t *opub, *osig, *odig, *expect;
} signjob;

static void* sign_worker(void* a) {
  signjob* j = (signjob*)a;
  EC_GROUP* grp = EC_GROUP_new_by_curve_name(NID_secp256k1);
  BIGNUM *n = NULL, *half = BN_new(), *d = BN_new();
  BN_hex2bn(&n, N_HEX); BN_rshift1(half, n);
  /* fixed-base precomputation makes OpenSSL's k*G several times faster */
  BN_CTX* bctx = BN_CTX_new();
  EC_GROUP_precompute_mult(grp, bctx);
  EC_KEY* key = EC_KEY_new();
  EC_KEY_set_group(key, grp);
  const BIGNUM *r, *s;
  BIGNUM* s2 = BN_new();
  for (size_t i = j->lo; i < j->hi; ++i) {
    size_t k = j->kidx ? j->kidx[i] : i % j->nkeys;
    uint8_t* dig = j->odig + 32 * i;
    if (j->msgdig) memcpy(dig, j->msgdig + 32 * i, 32);
    else {
      uint8_t m[24]; memcpy(m, "gv-dig", 6);
      for (int q = 0; q < 8; ++q) { m[6 + q] = (uint8_t)(j->seed >> (8 * q)); m[14 + q] = (uint8_t)((uint64_t)i >> (8 * q)); }
      m[22] = m[23] = 0;
      SHA256(m, sizeof m, dig);
    }
    BN_bin2bn(j->priv + 32 * k, 32, d);
    EC_KEY_set_private_key(key, d);
    ECDSA_SIG* sg = ECDSA_do_sign(dig, 32, key);
    ECDSA_SIG_get0(sg, &r, &s);
    if (BN_cmp(s, half) > 0) { BN_sub(s2, n, s); } else { BN_copy(s2, s); }
    uint8_t* sig = j->osig + 64 * i;
    BN_bn2binpad(r, sig, 32); BN_bn2binpad(s2, sig + 32, 32);
    ECDSA_SIG_free(sg);
    memcpy(j->opub + 33 * i, j->pub + 33 * k, 33);
    j->expect[i] = 1;
    /* adversarial mutation (C3): split evenly over six rejection classes */
    uint64_t st = j->seed ^ (0xA5A5A5A5ULL * (i + 1));
    uint64_t u = splitmix(&st);
    if ((double)(u >> 11) * (1.0 / 9007199254740992.0) < j->adv) {
      uint64_t v = splitmix(&st);
      j->expect[i] = 0;
      switch (v % 6) {
        case 0: { /* high-S */ BIGNUM* t = BN_new(); BN_bin2bn(sig + 32, 32, t); BN_sub(t, n, t); BN_bn2binpad(t, sig + 32, 32); BN_free(t); break; }
        case 1: { /* r >= n */ BIGNUM* t = BN_new(); BN_copy(t, n); BN_add_word(t, (unsigned)(v >> 40) & 0xFFFF); BN_bn2binpad(t, sig, 32); BN_free(t); break; }
        case 2: /* s == 0 or huge */ memset(sig + 32, (v >> 8) & 1 ? 0xFF : 0x00, 32); break;
        case 3: /* random x (off-curve or wrong key) */ for (int q = 1; q < 33; ++q) j->opub[33 * i + q] = (uint8_t)splitmix(&st); break;
        case 4: { static const uint8_t bad[7] = {0, 1, 4, 5, 6, 7, 0xFF}; j->opub[33 * i] = bad[(v >> 8) % 7]; break; }
        default: /* wrong message */ dig[(v >> 8) & 31] ^= (uint8_t)(1u << ((v >> 16) & 7)); break;
      }
    }
  }
  BN_free(s2); EC_KEY_free(key); BN_free(n); BN_free(half); BN_free(d); BN_CTX_free(bctx); EC_GROUP_free(grp);
  return NULL;
}

/* n signed items over digests.  Item i uses key kidx[i] (or i % nkeys when
 * kidx is NULL); digest = SHA256("gv-dig"||seed||i) unless msgdig (n x 32) is
 * given (message path: the caller hashed the sign bytes).  adv in [0,1): the
 * fraction of items mutated into invalid ones.  expect[i] = 1 valid, 0 invalid. */
int gvw_sign(size_t n, uint64_t seed, size_t nkeys, const uint8_t* priv32, const uint8_t* pub33,
             const uint32_t* kidx, const uint8_t* msgdig, double adv, uint8_t* out_pub33,
             uint8_t* out_sig64, uint8_t* out_dig32, uint8_t* expect, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256]; signjob js[256];
  for (int t = 0; t < threads; ++t) {
    signjob j = {n * t / threads, n * (t + 1) / threads, nkeys, seed, adv, priv32, pub33, kidx, msgdig,
                 out_pub33, out_sig64, out_dig32, expect};
    js[t] = j;
    pthread_create(&th[t], NULL, sign_worker, &js[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  return 0;
}

/* C1/C4 sign bytes: StdSignBytes(MsgSend) for account i (from key i to key
 * (i+1) % nkeys), accnum = i, sequence = seq.  Writes into blob (capacity
 * blob_cap) with off/len per item; returns total bytes or -1 on overflow. */
long long gvw_msgsend_signbytes(size_t n, const uint8_t* pub33, size_t nkeys, uint64_t seq,
                                uint8_t* blob, size_t blob_cap, uint64_t* off, uint32_t* len) {
  size_t pos = 0;
  char from[64], to[64];
  for (size_t i = 0; i < n; ++i) {
    uint8_t h[32], a1[20], a2[20];
    SHA256(pub33 + 33 * (i % nkeys), 33, h); ripemd160_32(h, a1);
    SHA256(pub33 + 33 * ((i + 1) % nkeys), 33, h); ripemd160_32(h, a2);
    bech32_cosmos(a1, from); bech32_cosmos(a2, to);
    char buf[1024];
    int m = snprintf(buf, sizeof buf,
      "{\"account_number\":\"%zu\",\"chain_id\":\"gv-bench\",\"fee\":{\"amount\":[{\"amount\":\"0\",\"denom\":\"stake\"}],"
      "\"gas\":\"1000000\"},\"memo\":\"\",\"msgs\":[{\"type\":\"cosmos-sdk/MsgSend\",\"value\":{\"amount\":"
      "[{\"amount\":\"10\",\"denom\":\"foocoin\"}],\"from_address\":\"%s\",\"to_address\":\"%s\"}}],\"sequence\":\"%llu\"}",
      i % nkeys, from, to, (unsigned long long)seq);
    if (pos + (size_t)m > blob_cap) return -1;
    memcpy(blob + pos, buf, (size_t)m);
    off[i] = pos; len[i] = (uint32_t)m; pos += (size_t)m;
  }
  return (long long)pos;
}

/* sha256 of every message (used to feed gvw_sign on the message path) */
void gvw_sha256_msgs(size_t n, const uint8_t* blob, const uint64_t* off, const uint32_t* len, uint8_t* out32) {
  for (size_t i = 0; i < n; ++i) SHA256(blob + off[i], len[i], out32 + 32 * i);
}

/* ----------------------------------------------- OpenSSL CPU baseline (iii)
 * SURVEY.md §8d "CPU timing beside it" (iii): tendermint VerifyBytes semantics
 * on OpenSSL 3 libcrypto -- the third CPU line next to the oracle port.  Per
 * item: btcec.ParsePubKey of the 33-byte SEC1 key (EC_POINT_oct2point: prefix
 * 02/03, x < p, square root exists), tendermint's low-S rule (s <= n/2,
 * secp256k1_nocgo.go), then ECDSA_do_verify (0 < r, s < n; x(u1*G + u2*Q)
 * mod n == r).  dig32 != NULL: items are digests; otherwise SHA-256 of
 * blob[off[i] .. off[i] + len[i]) is taken first (the full VerifyBytes).
 * ok[i] = 1 / 0.  Timed by bench.py; not the oracle, not the product. */
typedef struct {
  size_t lo, hi;
  const uint8_t *pub, *sig, *dig, *blob; const uint64_t* off; const uint32_t* len;
  uint8_t* ok;
} verjob;

static void* verify_worker(void* a) {
  verjob* j = (verjob*)a;
  EC_GROUP* grp = EC_GROUP_new_by_curve_name(NID_secp256k1);
  BN_CTX* bctx = BN_CTX_new();
  EC_GROUP_precompute_mult(grp, bctx);
  BIGNUM *n = NULL, *half = BN_new();
  BN_hex2bn(&n, N_HEX); BN_rshift1(half, n);
  EC_KEY* key = EC_KEY_new();
  EC_KEY_set_group(key, grp);
  EC_POINT* pt = EC_POINT_new(grp);
  for (size_t i = j->lo; i < j->hi; ++i) {
    uint8_t h[32];
    const uint8_t* e = j->dig ? j->dig + 32 * i : h;
    if (!j->dig) SHA256(j->blob + j->off[i], j->len[i], h);
    int ok = 0;
    if (EC_POINT_oct2point(grp, pt, j->pub + 33 * i, 33, bctx) == 1 && EC_KEY_set_public_key(key, pt) == 1) {
      BIGNUM* r = BN_bin2bn(j->sig + 64 * i, 32, NULL);
      BIGNUM* s = BN_bin2bn(j->sig + 64 * i + 32, 32, NULL);
      if (BN_cmp(s, half) <= 0) {
        ECDSA_SIG* sg = ECDSA_SIG_new();
        ECDSA_SIG_set0(sg, r, s);            /* takes ownership */
        ok = ECDSA_do_verify(e, 32, sg, key) == 1;
        ECDSA_SIG_free(sg);
      } else {
        BN_free(r); BN_free(s);
      }
    }
    j->ok[i] = (uint8_t)ok;
  }
  EC_POINT_free(pt); EC_KEY_free(key); BN_free(n); BN_free(half); BN_CTX_free(bctx); EC_GROUP_free(grp);
  return NULL;
}

int gvw_openssl_verify(size_t n, const uint8_t* pub33, const uint8_t* sig64, const uint8_t* dig32,
                       const uint8_t* blob, const uint64_t* off, const uint32_t* len, uint8_t* ok, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256]; verjob js[256];
  for (int t = 0; t < threads; ++t) {
    verjob j = {n * t / threads, n * (t + 1) / threads, pub33, sig64, dig32, blob, off, len, ok};
    js[t] = j;
    pthread_create(&th[t], NULL, verify_worker, &js[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  return 0;
}

/* single-item helpers for the client-side tx kit (cosmos-sdk-rootchain_amd/txkit.py) */
int gvw_pubkey(const uint8_t priv32[32], uint8_t pub33[33]) {
  EC_GROUP* grp = EC_GROUP_new_by_curve_name(NID_secp256k1);
  BN_CTX* ctx = BN_CTX_new();
  BIGNUM* d = BN_bin2bn(priv32, 32, NULL);
  EC_POINT* pt = EC_POINT_new(grp);
  int ok = EC_POINT_mul(grp, pt, d, NULL, NULL, ctx) == 1 &&
           EC_POINT_point2oct(grp, pt, POINT_CONVERSION_COMPRESSED, pub33, 33, ctx) == 33;
  EC_POINT_free(pt); BN_free(d); BN_CTX_free(ctx); EC_GROUP_free(grp);
  return ok ? 0 : -1;
}

/* ECDSA over a 32-byte digest, low-S normalised (tendermint Sign): R||S */
int gvw_sign_digest(const uint8_t priv32[32], const uint8_t dig32[32], uint8_t sig64[64]) {
  EC_KEY* key = EC_KEY_new_by_curve_name(NID_secp256k1);
  BIGNUM *d = BN_bin2bn(priv32, 32, NULL), *n = NULL, *half = BN_new(), *s2 = BN_new();
  BN_hex2bn(&n, N_HEX); BN_rshift1(half, n);
  EC_KEY_set_private_key(key, d);
  ECDSA_SIG* sg = ECDSA_do_sign(dig32, 32, key);
  int rc = -1;
  if (sg) {
    const BIGNUM *r, *s;
    ECDSA_SIG_get0(sg, &r, &s);
    if (BN_cmp(s, half) > 0) BN_sub(s2, n, s); else BN_copy(s2, s);
    BN_bn2binpad(r, sig64, 32); BN_bn2binpad(s2, sig64 + 32, 32);
    ECDSA_SIG_free(sg);
    rc = 0;
  }
  BN_free(d); BN_free(n); BN_free(half); BN_free(s2); EC_KEY_free(key);
  return rc;
}

/* ----------------------------------------------------------- C4 blocks */
/* C4 workload: ntx k-of-n multisig MsgSend txs as amino
 * StdTx bytes.  Tx t belongs to account a = t % nacct with sequence
 * t / nacct.  Per account the caller gives the constant pieces:
 *   sb_pre  StdSignBytes up to the sequence value ('..."sequence":"'),
 *   head    the tx bytes up to its first multisignature entry (StdTx prefix,
 *           msg, fee, StdSignature header, multisig pubkey, bit array),
 *   k, kidx[a*8 + j]  the keys (indices into priv32) of the k set bits.
 * This signs SHA256(sb_pre || seq || '"}') with each of the k keys and writes
 * head || k x (0x12 0x40 r || s) at out + off[t].
 * Signing speed: 8M OpenSSL ECDSA_do_sign calls take minutes, so each key
 * signs with ONE nonce k (R = k*G and k^-1 precomputed per key): every
 * signature is still a distinct valid low-S (r, s) over a distinct digest,
 * s = k^-1 (e + r d) mod n; verification work does not depend on the nonce.
 * (Nonce reuse would leak the key -- irrelevant for synthetic keys.) */
typedef struct { size_t lo, hi; const uint8_t* priv; uint8_t *r, *kinv, *rd; } c4key;
static void* c4_key_worker(void* arg) {
  c4key* j = (c4key*)arg;
  EC_GROUP* grp = EC_GROUP_new_by_curve_name(NID_secp256k1);
  BN_CTX* ctx = BN_CTX_new();
  EC_GROUP_precompute_mult(grp, ctx);
  BIGNUM *n = NULL, *k = BN_new(), *d = BN_new(), *r = BN_new(), *t = BN_new(), *x = BN_new();
  BN_hex2bn(&n, N_HEX);
  EC_POINT* R = EC_POINT_new(grp);
  for (size_t i = j->lo; i < j->hi; ++i) {
    uint8_t m[40], h[32];
    memcpy(m, j->priv + 32 * i, 32); memcpy(m + 32, "c4-nonce", 8);
    SHA256(m, sizeof m, h);
    BN_bin2bn(h, 32, k); BN_mod(k, k, n, ctx); if (BN_is_zero(k)) BN_one(k);
    EC_POINT_mul(grp, R, k, NULL, NULL, ctx);
    EC_POINT_get_affine_coordinates(grp, R, x, NULL, ctx);
    BN_nnmod(r, x, n, ctx);
    BN_bin2bn(j->priv + 32 * i, 32, d);
    BN_mod_mul(t, r, d, n, ctx);
    BN_bn2binpad(r, j->r + 32 * i, 32);
    BN_bn2binpad(t, j->rd + 32 * i, 32);
    BN_mod_inverse(t, k, n, ctx);
    BN_bn2binpad(t, j->kinv + 32 * i, 32);
  }
  EC_POINT_free(R); BN_free(n); BN_free(k); BN_free(d); BN_free(r); BN_free(t); BN_free(x);
  BN_CTX_free(ctx); EC_GROUP_free(grp);
  return NULL;
}

typedef struct {
  size_t lo, hi, nacct;
  const uint8_t *r, *kinv, *rd;
  const uint8_t* sbb; const uint64_t* sbo; const uint32_t* sbl;
  const uint8_t* hb; const uint64_t* ho; const uint32_t* hl;
  const uint8_t* k; const uint32_t* kidx;
  const uint64_t* off; uint8_t* out;
} c4job;

static void* c4_worker(void* arg) {
  c4job* j = (c4job*)arg;
  BN_CTX* ctx = BN_CTX_new();
  BIGNUM *n = NULL, *half = BN_new(), *e = BN_new(), *a = BN_new(), *ki = BN_new(), *s = BN_new();
  BN_hex2bn(&n, N_HEX); BN_rshift1(half, n);
  char seq[32];
  for (size_t t = j->lo; t < j->hi; ++t) {
    size_t ac = t % j->nacct;
    int ns = snprintf(seq, sizeof seq, "%llu\"}", (unsigned long long)(t / j->nacct));
    SHA256_CTX c; uint8_t dig[32];
    SHA256_Init(&c); SHA256_Update(&c, j->sbb + j->sbo[ac], j->sbl[ac]); SHA256_Update(&c, seq, (size_t)ns);
    SHA256_Final(dig, &c);
    uint8_t* o = j->out + j->off[t];
    memcpy(o, j->hb + j->ho[ac], j->hl[ac]);
    o += j->hl[ac];
    BN_bin2bn(dig, 32, e);                         /* hashToInt: 32-byte digest, no truncation */
    for (int q = 0; q < j->k[ac]; ++q) {
      const size_t key = j->kidx[ac * 8 + q];
      BN_bin2bn(j->rd + 32 * key, 32, a);
      BN_mod_add(a, a, e, n, ctx);                 /* e + r d */
      BN_bin2bn(j->kinv + 32 * key, 32, ki);
      BN_mod_mul(s, ki, a, n, ctx);                /* k^-1 (e + r d) */
      if (BN_cmp(s, half) > 0) BN_sub(s, n, s);    /* low-S (tendermint Sign) */
      o[0] = 0x12; o[1] = 0x40;
      memcpy(o + 2, j->r + 32 * key, 32);
      BN_bn2binpad(s, o + 34, 32);
      o += 66;
    }
  }
  BN_free(n); BN_free(half); BN_free(e); BN_free(a); BN_free(ki); BN_free(s); BN_CTX_free(ctx);
  return NULL;
}

int gvw_c4_txs(size_t ntx, size_t nacct, size_t nkeys, const uint8_t* priv32,
               const uint8_t* sb_blob, const uint64_t* sb_off, const uint32_t* sb_len,
               const uint8_t* head_blob, const uint64_t* head_off, const uint32_t* head_len,
               const uint8_t* k, const uint32_t* kidx, const uint64_t* tx_off, uint8_t* out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  uint8_t* r = malloc(32 * nkeys);
  uint8_t* kinv = malloc(32 * nkeys);
  uint8_t* rd = malloc(32 * nkeys);
  if (!r || !kinv || !rd) { free(r); free(kinv); free(rd); return -1; }
  pthread_t th[256];
  c4key ks[256];
  for (int t = 0; t < threads; ++t) {
    c4key kk = {nkeys * t / threads, nkeys * (t + 1) / threads, priv32, r, kinv, rd};
    ks[t] = kk;
    pthread_create(&th[t], NULL, c4_key_worker, &ks[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  c4job js[256];
  for (int t = 0; t < threads; ++t) {
    c4job jj = {ntx * t / threads, ntx * (t + 1) / threads, nacct, r, kinv, rd, sb_blob, sb_off, sb_len,
                head_blob, head_off, head_len, k, kidx, tx_off, out};
    js[t] = jj;
    pthread_create(&th[t], NULL, c4_worker, &js[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(r); free(kinv); free(rd);
  return 0;
}

/* ---- ed25519: OpenSSL Ed25519 (RFC 8032) signatures of
 * item i's message with key i % nkeys; pub_out = that key's 32 bytes. */
#include <openssl/evp.h>
typedef struct {
  size_t lo, hi, nkeys;
  EVP_PKEY** keys;
  const uint8_t* blob;
  const uint64_t* off;
  const uint32_t* len;
  uint8_t *pub, *sig;
  int err;
} ed_job;

static void* ed_worker(void* a) {
  ed_job* j = (ed_job*)a;
  EVP_MD_CTX* c = EVP_MD_CTX_new();
  for (size_t i = j->lo; i < j->hi && !j->err; ++i) {
    EVP_PKEY* k = j->keys[i % j->nkeys];
    size_t pl = 32, sl = 64;
    if (EVP_PKEY_get_raw_public_key(k, j->pub + i * 32, &pl) != 1 ||
        EVP_DigestSignInit(c, NULL, NULL, NULL, k) != 1 ||
        EVP_DigestSign(c, j->sig + i * 64, &sl, j->blob + j->off[i], j->len[i]) != 1)
      j->err = 1;
    EVP_MD_CTX_reset(c);
  }
  EVP_MD_CTX_free(c);
  return NULL;
}

int gvw_ed25519_sign(size_t n, size_t nkeys, const uint8_t* seeds32, const uint8_t* blob, const uint64_t* off,
                     const uint32_t* len, uint8_t* pub_out, uint8_t* sig_out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  EVP_PKEY** keys = (EVP_PKEY**)calloc(nkeys, sizeof(EVP_PKEY*));
  int rc = 0;
  for (size_t k = 0; k < nkeys && !rc; ++k)
    if (!(keys[k] = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, NULL, seeds32 + 32 * k, 32))) rc = -1;
  if (!rc) {
    pthread_t th[256];
    ed_job js[256];
    const size_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
      js[t] = (ed_job){(size_t)t * per < n ? (size_t)t * per : n, (size_t)(t + 1) * per < n ? (size_t)(t + 1) * per : n,
                       nkeys, keys, blob, off, len, pub_out, sig_out, 0};
      pthread_create(&th[t], NULL, ed_worker, &js[t]);
    }
    for (int t = 0; t < threads; ++t) {
      pthread_join(th[t], NULL);
      if (js[t].err) rc = -2;
    }
  }
  for (size_t k = 0; k < nkeys; ++k)
    if (keys[k]) EVP_PKEY_free(keys[k]);
  free(keys);
  return rc;
}

/* OpenSSL Ed25519 verify of n items (the CPU line beside the GPU's ed25519
 * rate; OpenSSL agrees with go1.14 crypto/ed25519 on canonical inputs). */
typedef struct {
  size_t lo, hi;
  const uint8_t *pub, *sig, *blob;
  const uint64_t* off;
  const uint32_t* len;
  uint8_t* out;
} edv_job;

static void* edv_worker(void* a) {
  edv_job* j = (edv_job*)a;
  EVP_MD_CTX* c = EVP_MD_CTX_new();
  for (size_t i = j->lo; i < j->hi; ++i) {
    EVP_PKEY* k = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, NULL, j->pub + i * 32, 32);
    j->out[i] = k && EVP_DigestVerifyInit(c, NULL, NULL, NULL, k) == 1 &&
                EVP_DigestVerify(c, j->sig + i * 64, 64, j->blob + j->off[i], j->len[i]) == 1;
    EVP_PKEY_free(k);
    EVP_MD_CTX_reset(c);
  }
  EVP_MD_CTX_free(c);
  return NULL;
}

int gvw_ed25519_verify(size_t n, const uint8_t* pub, const uint8_t* sig, const uint8_t* blob, const uint64_t* off,
                       const uint32_t* len, uint8_t* out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  edv_job js[256];
  const size_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    js[t] = (edv_job){(size_t)t * per < n ? (size_t)t * per : n, (size_t)(t + 1) * per < n ? (size_t)(t + 1) * per : n,
                      pub, sig, blob, off, len, out};
    pthread_create(&th[t], NULL, edv_worker, &js[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  return 0;
}
