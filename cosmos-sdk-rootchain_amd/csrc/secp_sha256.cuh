// secp_sha256.cuh -- SHA-256 on gfx950, one message per lane.
// Restates tendermint crypto.Sha256 -> Go crypto/sha256.Sum256 (FIPS 180-4)
// as used by VerifyBytes (tendermint v0.33.4 secp256k1_nocgo.go) over the
// StdSignBytes produced at x/auth/types/stdtx.go:248-259.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gv {

// Round constants as compile-time literals: with the rounds unrolled every
// K[i] becomes an instruction immediate (a __constant__ table costs one scalar
// memory load -- and its wait -- per round: 229 -> ~95 cycles per round on a
// lone wave, tools/microbench/fsl_check.hip).
struct Sha256K {
  static constexpr uint32_t k[64] = {
  0x428a2f98u,0x71374491u,0xb5c0fbcfu,0xe9b5dba5u,0x3956c25bu,0x59f111f1u,0x923f82a4u,0xab1c5ed5u,
  0xd807aa98u,0x12835b01u,0x243185beu,0x550c7dc3u,0x72be5d74u,0x80deb1feu,0x9bdc06a7u,0xc19bf174u,
  0xe49b69c1u,0xefbe4786u,0x0fc19dc6u,0x240ca1ccu,0x2de92c6fu,0x4a7484aau,0x5cb0a9dcu,0x76f988dau,
  0x983e5152u,0xa831c66du,0xb00327c8u,0xbf597fc7u,0xc6e00bf3u,0xd5a79147u,0x06ca6351u,0x14292967u,
  0x27b70a85u,0x2e1b2138u,0x4d2c6dfcu,0x53380d13u,0x650a7354u,0x766a0abbu,0x81c2c92eu,0x92722c85u,
  0xa2bfe8a1u,0xa81a664bu,0xc24b8b70u,0xc76c51a3u,0xd192e819u,0xd6990624u,0xf40e3585u,0x106aa070u,
  0x19a4c116u,0x1e376c08u,0x2748774cu,0x34b0bcb5u,0x391c0cb3u,0x4ed8aa4au,0x5b9cca4fu,0x682e6ff3u,
  0x748f82eeu,0x78a5636fu,0x84c87814u,0x8cc70208u,0x90befffau,0xa4506cebu,0xbef9a3f7u,0xc67178f2u};
};

__device__ __forceinline__ uint32_t sha_rotr(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}

// One compression of the 16-word big-endian block w[] into h[].
__device__ __forceinline__ void sha256_compress(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = sha_rotr(w15, 7) ^ sha_rotr(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = sha_rotr(w2, 17) ^ sha_rotr(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = sha_rotr(e, 6) ^ sha_rotr(e, 11) ^ sha_rotr(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = hh + S1 + ch + Sha256K::k[i] + wi;
    uint32_t S0 = sha_rotr(a, 2) ^ sha_rotr(a, 13) ^ sha_rotr(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// SHA-256 of msg[0..len) read from global memory; out = 8 big-endian words.
__device__ __forceinline__ void sha256_msg(uint32_t out[8], const uint8_t* msg, uint32_t len) {
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const uint32_t nblocks = (len + 9u + 63u) >> 6;
  const uint64_t bitlen = (uint64_t)len * 8u;
  for (uint32_t blk = 0; blk < nblocks; ++blk) {
    uint32_t w[16];
    const uint32_t base = blk << 6;
    if (base + 64u <= len) {
      // full data block: whole words
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint8_t* p = msg + base + 4 * j;
        w[j] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        uint32_t word = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t pos = base + 4 * j + k;
          uint32_t byte;
          if (pos < len) byte = msg[pos];
          else if (pos == len) byte = 0x80u;
          else byte = 0u;
          word = (word << 8) | byte;
        }
        w[j] = word;
      }
      if (blk == nblocks - 1) {
        w[14] = (uint32_t)(bitlen >> 32);
        w[15] = (uint32_t)bitlen;
      }
    }
    sha256_compress(h, w);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = h[i];
}

// SHA-256 of ONE message by a whole wave (the sliced small-batch kernels'
// scalar wave: every lane passes the same msg / len).  The padded message is
// read 256 bytes at a time, one big-endian word per lane (byte loads: the
// message may sit at any offset, e.g. in pinned host memory read zero-copy),
// the next chunk's loads issued before the current chunk's compressions; a
// block's 16 words come out of the lanes with readlane and the rounds run on
// the VALU (values pinned to VGPRs).  out = 8 big-endian state words.
__device__ __forceinline__ uint32_t sha256_wave_word(const uint8_t* msg, uint32_t len, uint32_t nb, uint32_t gw) {
  const uint64_t bitlen = (uint64_t)len * 8u;
  if (gw == 16u * (nb - 1u) + 14u) return (uint32_t)(bitlen >> 32);
  if (gw == 16u * (nb - 1u) + 15u) return (uint32_t)bitlen;
  uint32_t word = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t pos = 4u * gw + (uint32_t)k;
    const uint32_t byte = pos < len ? msg[pos] : (pos == len ? 0x80u : 0u);
    word = (word << 8) | byte;
  }
  return word;
}
__device__ __forceinline__ void sha256_msg_wave(uint32_t out[8], const uint8_t* msg, uint32_t len) {
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const uint32_t lane = __lane_id();
#pragma unroll
  for (int i = 0; i < 8; ++i) asm("" : "+v"(h[i]));
  const uint32_t nb = (len + 9u + 63u) >> 6;
  const uint32_t nchunks = (nb + 3u) >> 2;
  uint32_t cur = sha256_wave_word(msg, len, nb, lane);
#pragma unroll 1
  for (uint32_t c = 0; c < nchunks; ++c) {
    const uint32_t nxt = c + 1u < nchunks ? sha256_wave_word(msg, len, nb, 64u * (c + 1u) + lane) : 0u;
    const uint32_t blocks = nb - 4u * c < 4u ? nb - 4u * c : 4u;
#pragma unroll 1
    for (uint32_t b = 0; b < blocks; ++b) {
      uint32_t w[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        w[j] = (uint32_t)__builtin_amdgcn_readlane((int)cur, (int)(16u * b + (uint32_t)j));
        asm("" : "+v"(w[j]));   // keep the rounds on the VALU: as scalar code every v_alignbit
      }                         // rotation costs a round trip through v_readfirstlane
      sha256_compress(h, w);
    }
    cur = nxt;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = h[i];
}

}  // namespace gv
