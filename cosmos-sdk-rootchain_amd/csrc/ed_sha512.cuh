// ed_sha512.cuh -- SHA-512 (FIPS 180-4), one message per lane, for the
// ed25519 challenge h = SHA-512(R || A || M) (go1.14 crypto/ed25519 Verify:
// h.Write(sig[:32]); h.Write(publicKey); h.Write(message)).
// Host-compilable (tests/test_ed_host.py builds it with g++).
#pragma once
#include <stdint.h>
#ifndef GV_DEV
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GV_DEV __device__ __forceinline__
#else
#define GV_DEV static inline
#endif
#endif
#ifndef GV_EDC
#if defined(__HIPCC__)
#define GV_EDC __constant__ const
#else
#define GV_EDC static const
#endif
#endif

namespace gv {
namespace ed {

GV_EDC uint64_t kSha512K[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

GV_DEV uint64_t sha512_rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

GV_DEV void sha512_compress(uint64_t h[8], uint64_t w[16]) {
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 80; ++i) {
    uint64_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint64_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const uint64_t s0 = sha512_rotr(w15, 1) ^ sha512_rotr(w15, 8) ^ (w15 >> 7);
      const uint64_t s1 = sha512_rotr(w2, 19) ^ sha512_rotr(w2, 61) ^ (w2 >> 6);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    const uint64_t S1 = sha512_rotr(e, 14) ^ sha512_rotr(e, 18) ^ sha512_rotr(e, 41);
    const uint64_t ch = (e & f) ^ (~e & g);
    const uint64_t t1 = hh + S1 + ch + kSha512K[i] + wi;
    const uint64_t S0 = sha512_rotr(a, 28) ^ sha512_rotr(a, 34) ^ sha512_rotr(a, 39);
    const uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// SHA-512(pre[0..64) || msg[0..len)) where pre is 16 little-endian words
// (bytes 4k..4k+3 in word k) and msg(i) returns byte i of the message.
// out = the 64-byte digest as 16 little-endian words (digest bytes 4k..4k+3),
// i.e. the integer ScReduce reads.
template <class Msg>
GV_DEV void sha512_pre64(uint32_t out[16], const uint32_t pre[16], Msg msg, uint32_t len) {
  uint64_t h[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull, 0xa54ff53a5f1d36f1ull,
                   0x510e527fade682d1ull, 0x9b05688c2b3e6c1full, 0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
  const uint32_t total = 64u + len;
  const uint32_t nblocks = (total + 17u + 127u) >> 7;
  for (uint32_t blk = 0; blk < nblocks; ++blk) {
    uint64_t w[16];
    const uint32_t base = blk << 7;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t p0 = base + 8u * (uint32_t)j;
      uint64_t word;
      if (p0 + 8u <= 64u) {                    // inside R || A: two pre words, big-endian
        const uint32_t lo = pre[p0 >> 2], hi = pre[(p0 >> 2) + 1];
        const uint32_t blo = __builtin_bswap32(lo), bhi = __builtin_bswap32(hi);
        word = ((uint64_t)blo << 32) | bhi;
      } else if (p0 >= 64u && p0 + 8u <= total) {   // whole word of message bytes
        word = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) word = (word << 8) | msg(p0 - 64u + (uint32_t)k);
      } else {                                 // message tail, padding, length
        word = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t pos = p0 + (uint32_t)k;
          uint32_t byte = 0;
          if (pos < total) byte = msg(pos - 64u);
          else if (pos == total) byte = 0x80u;
          word = (word << 8) | byte;
        }
      }
      w[j] = word;
    }
    if (blk == nblocks - 1) {                  // 128-bit big-endian bit length (high half 0)
      w[14] = 0;
      w[15] = (uint64_t)total * 8u;
    }
    sha512_compress(h, w);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    out[2 * i] = __builtin_bswap32((uint32_t)(h[i] >> 32));
    out[2 * i + 1] = __builtin_bswap32((uint32_t)h[i]);
  }
}

}  // namespace ed
}  // namespace gv
