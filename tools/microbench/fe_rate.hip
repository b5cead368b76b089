// Field-layer throughput on gfx950: 8 x 32 (inline-asm carry chains,
// secp_field.cuh) vs 10 x 26 reduced radix (secp_field26.cuh).  Each lane runs
// a dependent chain of ITERS operations; the grid holds many waves per SIMD
// (occupancy set by the kernel's VGPRs, as in k_ecmult).  Results of the two
// representations are cross-checked (mismatch count printed).
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_group.cuh"
#include "../field26/secp_field26.cuh"
#include <stdio.h>

using namespace gv;
#define ITERS 512
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ void seed_fe(fe& a, u32 g, u32 s) {
  u32 x = g * 2654435761u + s;
  for (int i = 0; i < 8; ++i) { x = x * 1664525u + 1013904223u; a.v[i] = x; }
  a.v[7] &= 0x7FFFFFFFu;
}

__global__ __launch_bounds__(256) void k_mul32(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b; seed_fe(a, g, s); seed_fe(b, g, s + 1);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) { fe_mul(a, a, b); fe_mul(b, b, a); }
  fe_normalize(a);
  for (int i = 0; i < 8; ++i) out[(size_t)i * gridDim.x * blockDim.x + g] = a.v[i];
}
__global__ __launch_bounds__(256) void k_mul26(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a0, b0; seed_fe(a0, g, s); seed_fe(b0, g, s + 1);
  fe26 a, b; fe26_from_words(a, a0.v); fe26_from_words(b, b0.v);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) { fe26_mul(a, a, b); fe26_mul(b, b, a); }
  u32 w[8]; fe26_to_words(w, a);
  for (int i = 0; i < 8; ++i) out[(size_t)i * gridDim.x * blockDim.x + g] = w[i];
}
__global__ __launch_bounds__(256) void k_sqr32(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b; seed_fe(a, g, s); seed_fe(b, g, s + 1);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) { fe_sqr(a, a); fe_sqr(b, b); }
  fe_add(a, a, b); fe_normalize(a);
  for (int i = 0; i < 8; ++i) out[(size_t)i * gridDim.x * blockDim.x + g] = a.v[i];
}
__global__ __launch_bounds__(256) void k_sqr26(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a0, b0; seed_fe(a0, g, s); seed_fe(b0, g, s + 1);
  fe26 a, b; fe26_from_words(a, a0.v); fe26_from_words(b, b0.v);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) { fe26_sqr(a, a); fe26_sqr(b, b); }
  fe26_add(a, a, b);
  u32 w[8]; fe26_to_words(w, a);
  for (int i = 0; i < 8; ++i) out[(size_t)i * gridDim.x * blockDim.x + g] = w[i];
}

// ---- point doubling: 8x32 dbl-2009-l (2M+5S) vs 10x26 3M+4S
struct gej26 { fe26 x, y, z; };
// in: X <= 10, Y <= 10, Z <= 2; out: X 10, Y 10, Z 2
__device__ __forceinline__ void gej26_double(gej26& r, const gej26& a) {
  fe26 A, B, C, D, E, t;
  fe26_sqr(A, a.x);                 // 1
  fe26_sqr(B, a.y);                 // 1
  fe26_mul(t, a.y, a.z);
  fe26_add(r.z, t, t);              // Z3 = 2YZ: 2
  fe26_sqr(C, B);                   // 1
  fe26_mul(D, a.x, B);              // 1
  fe26_mul_int(E, A, 3);            // 3
  fe26_sqr(t, E);                   // F: 1
  fe26_mul_int(A, D, 8);            // 8D: 8
  fe26_sub(r.x, t, A, 8);           // X3 = F - 8D: 10
  fe26_mul_int(D, D, 4);            // 4
  fe26_sub(t, D, r.x, 10);          // 4D - X3: 15
  fe26_mul(t, E, t);                // 1
  fe26_mul_int(C, C, 8);            // 8
  fe26_sub(r.y, t, C, 8);           // 10
}

__global__ __launch_bounds__(256) void k_dbl32(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  gej p; seed_fe(p.x, g, s); seed_fe(p.y, g, s + 1); seed_fe(p.z, g, s + 2);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) gej_double(p, p);
  fe_normalize(p.x); fe_normalize(p.y); fe_normalize(p.z);
  const size_t C = (size_t)gridDim.x * blockDim.x;
  for (int i = 0; i < 8; ++i) { out[i * C + g] = p.x.v[i]; out[(8 + i) * C + g] = p.y.v[i]; out[(16 + i) * C + g] = p.z.v[i]; }
}
__global__ __launch_bounds__(256) void k_dbl26(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  fe x, y, z; seed_fe(x, g, s); seed_fe(y, g, s + 1); seed_fe(z, g, s + 2);
  gej26 p; fe26_from_words(p.x, x.v); fe26_from_words(p.y, y.v); fe26_from_words(p.z, z.v);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) gej26_double(p, p);
  u32 wx[8], wy[8], wz[8];
  fe26_to_words(wx, p.x); fe26_to_words(wy, p.y); fe26_to_words(wz, p.z);
  const size_t C = (size_t)gridDim.x * blockDim.x;
  for (int i = 0; i < 8; ++i) { out[i * C + g] = wx[i]; out[(8 + i) * C + g] = wy[i]; out[(16 + i) * C + g] = wz[i]; }
}

typedef void (*kfn)(u32*, u32);
static int run(const char* name, kfn f, int blocks, u32* d, double ops_per_lane, float* ms_out) {
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, 5u);
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, 5u);
    CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
  }
  const double lanes = (double)blocks * 256;
  printf("{\"kernel\": \"%s\", \"ms\": %.3f, \"ops_per_s\": %.4e, \"ns_per_op_per_lane\": %.3f}\n", name, best,
         lanes * ops_per_lane / (best * 1e-3), best * 1e6 / (lanes * ops_per_lane) * lanes / 1e6);
  *ms_out = best;
  return 0;
}

static int cmp(const char* what, u32* d0, u32* d1, size_t words) {
  u32* h0 = (u32*)malloc(words * 4); u32* h1 = (u32*)malloc(words * 4);
  if (hipMemcpy(h0, d0, words * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  if (hipMemcpy(h1, d1, words * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  size_t bad = 0;
  for (size_t i = 0; i < words; ++i) bad += h0[i] != h1[i];
  printf("{\"check\": \"%s\", \"mismatched_words\": %zu, \"words\": %zu}\n", what, bad, words);
  free(h0); free(h1);
  return 0;
}

int main() {
  const int blocks = 256 * 8;          // 2048 blocks x 256 = 524288 lanes
  const size_t lanes = (size_t)blocks * 256;
  u32 *d0, *d1;
  CHK(hipMalloc(&d0, lanes * 24 * 4)); CHK(hipMalloc(&d1, lanes * 24 * 4));
  float ms;
  if (run("fe_mul 8x32", k_mul32, blocks, d0, 2.0 * ITERS, &ms)) return 1;
  if (run("fe_mul 10x26", k_mul26, blocks, d1, 2.0 * ITERS, &ms)) return 1;
  if (cmp("mul", d0, d1, lanes * 8)) return 1;
  if (run("fe_sqr 8x32", k_sqr32, blocks, d0, 2.0 * ITERS, &ms)) return 1;
  if (run("fe_sqr 10x26", k_sqr26, blocks, d1, 2.0 * ITERS, &ms)) return 1;
  if (cmp("sqr", d0, d1, lanes * 8)) return 1;
  if (run("gej_double 8x32 (2M+5S)", k_dbl32, blocks, d0, ITERS, &ms)) return 1;
  if (run("gej_double 10x26 (3M+4S)", k_dbl26, blocks, d1, ITERS, &ms)) return 1;
  if (cmp("dbl", d0, d1, lanes * 24)) return 1;
  return 0;
}
