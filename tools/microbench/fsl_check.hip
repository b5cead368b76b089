// Limb-sliced field layer (csrc/secp_fsl.cuh) against the one-lane 9 x 29
// layer: products, mul_plus, mul2, norm/sub, doubling and the scaled mixed
// addition, chained so that every output feeds the next operation (bounds are
// exercised at their own fixed points), plus single-wave latency of the
// sliced ops.  Prints one JSON line: mismatches per op and microseconds per op.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DF29_NCH=2 -DF29X_NCH=2 \
//         tools/microbench/fsl_check.hip -o tools/microbench/fsl_check
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_field.cuh"
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_group29.cuh"
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_group29x.cuh"
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_fsl.cuh"
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_modinv_sl.cuh"
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_scalar.cuh"
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_sha256.cuh"

using namespace gv;
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

enum { T_MUL, T_MULPLUS, T_MUL2, T_SUB, T_DBL, T_ADD, T_N };
static const char* kT[T_N] = {"mul", "mul_plus", "mul2", "sub", "double", "add_scaled"};

__device__ void seed(u32 w[8], u32 g, u32 s, int mode) {
  u32 x = g * 2654435761u + s * 40503u + 12345u;
  for (int i = 0; i < 8; ++i) { x = x * 1664525u + 1013904223u; w[i] = x ^ (x >> 13); }
  if (mode == 1) for (int i = 0; i < 8; ++i) w[i] = 0xFFFFFFFFu;               // 2^256 - 1
  if (mode == 2) { const u32 p[8] = {0xFFFFFC2Eu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                     0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};       // p - 1
                   for (int i = 0; i < 8; ++i) w[i] = p[i]; }
  if (mode == 3) for (int i = 0; i < 8; ++i) w[i] = i == 0 ? 1u : 0u;
}

GV_DEV bool same(u32 v, const fe29& s) {
  fe29 g;
  fsl_gather(g, v);
  u32 a[8], b[8];
  f29_to_words(a, g);
  f29_to_words(b, s);
  u32 d = 0;
  for (int i = 0; i < 8; ++i) d |= a[i] ^ b[i];
  return d == 0;
}

// one row per case; 4 rows per wave
__global__ __launch_bounds__(64) void k_check(int test, int iters, u32* bad) {
  const fslk k = fsl_consts();
  const u32 row = blockIdx.x * 4u + (threadIdx.x >> 4);
  const int mode = (int)(row % 7u) < 4 ? (int)(row % 7u) : 0;
  u32 wa[8], wb[8], wc[8];
  seed(wa, row, 1, mode); seed(wb, row, 2, mode == 3 ? 0 : mode); seed(wc, row, 3, 0);
  fe29 A, B, Cc;
  f29_from_words(A, wa); f29_from_words(B, wb); f29_from_words(Cc, wc);
  u32 a = fsl_scatter(A, k), b = fsl_scatter(B, k), c = fsl_scatter(Cc, k);
  u32 nbad = 0;
  if (test == T_MUL || test == T_MULPLUS || test == T_MUL2 || test == T_SUB) {
    for (int i = 0; i < iters; ++i) {
      if (test == T_MUL) {
        a = fsl_mul(a, b, k); f29_mul(A, A, B);
        b = fsl_sqr(b, k); f29_sqr(B, B);
      } else if (test == T_MULPLUS) {             // a b - 8c
        a = fsl_mul_plus(a, b, k.big8 - ((u64)c << 3), k);
        fe29 t, e; f29_mul(t, A, B); f29_shl_norm<3>(e, Cc); f29_sub_norm<1>(A, t, e);
        c = fsl_mul(c, a, k); f29_mul(Cc, Cc, A);
      } else if (test == T_MUL2) {                // a b + (-c) (4c + bias - a)
        const u32 t = (c << 2) + k.bias - a;
        const u32 nc = k.bias - c;
        const u32 r = fsl_mul2(b, t, nc, a, k);
        fe29 t4, tt, u1, u2, ncs;
        f29_shl_norm<2>(t4, Cc); f29_sub_norm<1>(tt, t4, A); f29_mul(u1, B, tt);
        f29_neg<1>(ncs, Cc); f29_mul(u2, ncs, A); f29_add(u1, u1, u2); f29_norm(u1, u1);
        a = c; A = Cc; c = r; Cc = u1;
      } else {                                    // sub / neg / norm chain
        a = fsl_sub(a, b, k); f29_sub_norm<1>(A, A, B);
        b = fsl_neg(a, k); f29_neg<1>(B, A); f29_norm(B, B);
        b = fsl_mul(b, c, k); f29_mul(B, B, Cc);
      }
      nbad += !same(a, A) || !same(b, B) || !same(c, Cc);
    }
  } else {
    gej29 P; P.x = A; P.y = B; P.z = Cc;
    gjsl Q; Q.x = a; Q.y = b; Q.z = c;
    bool pinf = false, qinf = false;
    for (int i = 0; i < iters; ++i) {
      if (test == T_DBL) {
        gej29x_double(P, P);
        gjsl_double(Q, Q, k);
      } else {
        // entry = (x, y) affine on the accumulator's curve; every 5th step the
        // accumulator itself (H == 0 -> doubling path), every 7th its negation
        fe29 x, y;
        u32 sx, sy;
        if (i % 5 == 4) {                          // x = X/Z^2 scaled: use az = Z -> H = 0
          x = P.x; y = P.y; f29_set_u32(P.z, 1); P.z = P.z;
          sx = Q.x; sy = Q.y;
          fe29 one; f29_set_u32(one, 1); Q.z = fsl_scatter(one, k); P.z = one;
          if (i % 7 == 3) { f29_neg<1>(y, y); sy = k.bias - sy; }
        } else {
          u32 w1[8], w2[8];
          seed(w1, row, 100 + i, 0); seed(w2, row, 200 + i, 0);
          f29_from_words(x, w1); f29_from_words(y, w2);
          sx = fsl_scatter(x, k); sy = fsl_scatter(y, k);
        }
        if (!pinf) gej29x_add_scaled(P, pinf, x, y, P.z);
        if (!qinf) gjsl_add_scaled(Q, qinf, sx, sy, Q.z, k);
        if (pinf != qinf) { nbad += 1; break; }
        if (pinf) break;
      }
      nbad += !same(Q.x, P.x) || !same(Q.y, P.y) || !same(Q.z, P.z);
    }
  }
  if ((threadIdx.x & 15u) == 0) atomicAdd(bad, nbad);
}

enum { L_MUL, L_SQRS, L_DBL, L_ADD, L_INV, L_GLV, L_SHAW, L_SHA1, L_N };
static const char* kL[L_N] = {"fsl_mul", "fsl_sqr", "gjsl_double", "gjsl_add_scaled", "s30_modinv_sl", "glv_split", "sha256_msg_wave_355B", "sha256_msg_lane_355B"};
static const int kLI[L_N] = {256, 256, 64, 64, 8, 32, 8, 8};

__global__ __launch_bounds__(64) void k_lat(int op, int iters, uint64_t* t, u32* sink, const uint8_t* msg) {
  const fslk k = fsl_consts();
  u32 w[8];
  seed(w, 0, 1, 0);
  fe29 A; f29_from_words(A, w);
  u32 a = fsl_scatter(A, k), b = a ^ 0x1234u;
  b &= k.m29;
  gjsl Q; Q.x = a; Q.y = b; Q.z = fsl_mul(a, b, k);
  bool inf = false;
  __syncthreads();
  const uint64_t w0 = wall_clock64(), c0 = clock64();
  switch (op) {
    case L_MUL:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) a = fsl_mul(a, b, k);
      break;
    case L_SQRS:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) a = fsl_sqr(a, k);
      break;
    case L_DBL:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) gjsl_double(Q, Q, k);
      break;
    case L_ADD:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) gjsl_add_scaled(Q, inf, a, b, Q.z, k);
      break;
    case L_INV:                                  // whole wave, the same scalar in every lane
#pragma unroll 1
      for (int i = 0; i < iters; ++i) {
        w[0] |= 1u;
        w[7] &= 0x7FFFFFFFu;
        s30_modinv_sl(w, w, k);
      }
      a ^= w[0];
      break;
    case L_SHAW:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) {
        u32 h[8];
        sha256_msg_wave(h, msg + (w[0] & 7u), 355);
        w[0] ^= h[0]; w[1] ^= h[7];
      }
      a ^= w[0];
      break;
    case L_SHA1:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) {
        u32 h[8];
        sha256_msg(h, msg + (w[0] & 7u), 355);
        w[0] ^= h[0]; w[1] ^= h[7];
      }
      a ^= w[0];
      break;
    case L_GLV:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) {
        u32 k1[4], k2[4], n1, n2;
        glv_split(k1, n1, k2, n2, w);
        w[0] ^= k1[0] ^ n1; w[1] ^= k2[1] ^ n2;
      }
      a ^= w[0];
      break;
  }
  const uint64_t c1 = clock64(), w1 = wall_clock64();
  sink[threadIdx.x] = a ^ Q.x ^ Q.y ^ Q.z ^ (u32)inf;
  if (threadIdx.x == 0) { t[0] = w1 - w0; t[1] = c1 - c0; }
}

int main() {
  u32* bad;
  uint64_t* dt;
  u32* sink;
  CHK(hipMalloc(&bad, 4));
  CHK(hipMalloc(&dt, 16));
  CHK(hipMalloc(&sink, 256));
  uint8_t* msg;
  CHK(hipMalloc(&msg, 1024));
  CHK(hipMemset(msg, 0x5A, 1024));
  printf("{\"mismatches\": {");
  for (int t = 0; t < T_N; ++t) {
    CHK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_check, dim3(256), dim3(64), 0, 0, t, 40, bad);
    CHK(hipDeviceSynchronize());
    u32 h;
    CHK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
    printf("%s\"%s\": %u", t ? ", " : "", kT[t], h);
  }
  printf("}, \"latency\": {");
  for (int op = 0; op < L_N; ++op) {
    double best = 1e30, cyc = 0;
    for (int rep = 0; rep < 5; ++rep) {
      hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, op, kLI[op], dt, sink, msg);
      CHK(hipDeviceSynchronize());
      uint64_t h[2];
      CHK(hipMemcpy(h, dt, 16, hipMemcpyDeviceToHost));
      const double us = h[0] * 0.01 / kLI[op];
      if (us < best) { best = us; cyc = (double)h[1] / kLI[op]; }
    }
    printf("%s\"%s\": {\"us\": %.4f, \"clk\": %.1f}", op ? ", " : "", kL[op], best, cyc);
  }
  printf("}}\n");
  return 0;
}
