// Single-wave latency of the latency kernels' building blocks (gv_lat.hip is
// built with F29_NCH = F29X_NCH = 2): one block of 64 threads, every op in a
// dependent chain, wall-clock (100 MHz) and shader-clock stamps around each
// loop.  Prints one JSON line: microseconds per op.  This is the cost model
// behind the C5 phase budget: a lone wave issues one
// instruction per ~4 cycles whatever the number of active lanes, so the
// latency of a phase is its instruction count on the critical lane.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DF29_NCH=2 -DF29X_NCH=2 \
//         tools/microbench/lat_ops.hip -o tools/microbench/lat_ops
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_field.cuh"
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_scalar.cuh"
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_group29.cuh"
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_group29x.cuh"
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_sc29.cuh"
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_modinv.cuh"

using namespace gv;
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

enum { OP_MUL, OP_SQR, OP_MULX, OP_DBL, OP_ADD, OP_MODINV, OP_SCMUL, OP_GLV, OP_SQRT, OP_FERMAT, OP_MODINV_VAR, OP_N };
static const char* kNames[OP_N] = {"f29_mul", "f29_sqr", "f29x_mul", "gej29x_double", "gej29x_add_scaled",
                                   "s30_modinv", "sc29_mul", "glv_split", "f29_sqrt_candidate", "sc29_inv", "s30_modinv_var"};
static const int kIters[OP_N] = {256, 256, 256, 64, 64, 8, 128, 32, 4, 4, 8};

__device__ void seed(u32 w[8], u32 g, u32 s) {
  u32 x = g * 2654435761u + s;
  for (int i = 0; i < 8; ++i) { x = x * 1664525u + 1013904223u; w[i] = x; }
  w[7] &= 0x7FFFFFFFu;
}

__global__ __launch_bounds__(64) void k_lat(int op, int iters, uint64_t* t, u32* sink) {
  const u32 g = threadIdx.x;
  u32 wa[8], wb[8];
  seed(wa, g, 1); seed(wb, g, 2);
  fe29 a, b;
  f29_from_words(a, wa); f29_from_words(b, wb);
  gej29 P; P.x = a; P.y = b; f29_set_u32(P.z, 1);
  bool inf = false;
  sc29 sa, sb;
  sc29_from_words(sa, wa); sc29_from_words(sb, wb);
  u32 acc = 0;
  __syncthreads();
  const uint64_t w0 = wall_clock64(), c0 = clock64();
  switch (op) {
    case OP_MUL:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) f29_mul(a, a, b);
      break;
    case OP_SQR:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) f29_sqr(a, a);
      break;
    case OP_MULX:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) f29x_mul(a, a, b);
      break;
    case OP_DBL:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) gej29x_double(P, P);
      break;
    case OP_ADD:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) gej29x_add_scaled(P, inf, a, b, P.z);
      break;
    case OP_MODINV:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) {
        wa[0] |= 1u;
        s30_modinv(wa, wa, [](bool done) { return __all(done) != 0; });
      }
      break;
    case OP_SCMUL:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) sc29_mul(sa, sa, sb);
      break;
    case OP_GLV:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) {
        u32 k1[4], k2[4], n1, n2;
        glv_split(k1, n1, k2, n2, wa);
        wa[0] ^= k1[0] ^ n1; wa[1] ^= k2[1] ^ n2;
      }
      break;
    case OP_SQRT:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) f29_sqrt_candidate(a, a);
      break;
    case OP_MODINV_VAR:
      if (g == 0) {                              // one lane, as in the sliced kernels
#pragma unroll 1
        for (int i = 0; i < iters; ++i) {
          wa[0] |= 1u;
          s30_modinv_var(wa, wa, []() {});
        }
      }
      break;
    case OP_FERMAT:
#pragma unroll 1
      for (int i = 0; i < iters; ++i) sc29_inv(sa, sa);
      break;
  }
  const uint64_t c1 = clock64(), w1 = wall_clock64();
  u32 o[8];
  f29_to_words(o, a);
  acc ^= o[0] ^ P.x.n[0] ^ P.z.n[3] ^ sa.n[0] ^ wa[0] ^ wa[1] ^ (u32)inf;
  sink[g] = acc;
  if (g == 0) { t[0] = w1 - w0; t[1] = c1 - c0; }
}

int main() {
  uint64_t* dt;
  u32* sink;
  CHK(hipMalloc(&dt, 16));
  CHK(hipMalloc(&sink, 256));
  printf("{");
  for (int op = 0; op < OP_N; ++op) {
    double best_us = 1e30, cyc = 0;
    for (int rep = 0; rep < 5; ++rep) {
      hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, op, kIters[op], dt, sink);
      CHK(hipDeviceSynchronize());
      uint64_t h[2];
      CHK(hipMemcpy(h, dt, 16, hipMemcpyDeviceToHost));
      const double us = h[0] * 0.01 / kIters[op];
      if (us < best_us) { best_us = us; cyc = (double)h[1] / kIters[op]; }
    }
    printf("%s\"%s\": {\"us\": %.4f, \"clk\": %.1f}", op ? ", " : "", kNames[op], best_us, cyc);
  }
  printf("}\n");
  return 0;
}
