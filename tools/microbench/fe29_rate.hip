// Field-layer throughput on gfx950: 8 x 32 (inline-asm carry chains,
// secp_field.cuh, the production layer) vs 9 x 29 reduced radix
// (secp_fe29.cuh).  Each lane runs a dependent chain of ITERS operations over
// a grid of many waves per SIMD.  Results of the two layers are cross-checked
// word for word (mismatch count printed).
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_group.cuh"
#include "../../cosmos-sdk-rootchain_amd/csrc/secp_fe29.cuh"
#include <stdio.h>
#include <stdlib.h>

using namespace gv;
#define ITERS 512
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ void seed_fe(fe& a, u32 g, u32 s) {
  u32 x = g * 2654435761u + s;
  for (int i = 0; i < 8; ++i) { x = x * 1664525u + 1013904223u; a.v[i] = x; }
  a.v[7] &= 0x7FFFFFFFu;
}
__device__ void put(u32* out, int row, u32 g, const u32 w[8]) {
  const size_t C = (size_t)gridDim.x * blockDim.x;
  for (int i = 0; i < 8; ++i) out[(row * 8 + i) * C + g] = w[i];
}

__global__ __launch_bounds__(256) void k_mul32(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b; seed_fe(a, g, s); seed_fe(b, g, s + 1);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) { fe_mul(a, a, b); fe_mul(b, b, a); }
  fe_normalize(a); put(out, 0, g, a.v);
}
__global__ __launch_bounds__(256) void k_mul29(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a0, b0; seed_fe(a0, g, s); seed_fe(b0, g, s + 1);
  fe29 a, b; f29_from_words(a, a0.v); f29_from_words(b, b0.v);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) { f29_mul(a, a, b); f29_mul(b, b, a); }
  u32 w[8]; f29_to_words(w, a); put(out, 0, g, w);
}
__global__ __launch_bounds__(256) void k_mul29x2(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a0, b0; seed_fe(a0, g, s); seed_fe(b0, g, s + 1);
  fe29 a, b; f29_from_words(a, a0.v); f29_from_words(b, b0.v);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) { f29_mulsqr<false, 2>(a, a, b); f29_mulsqr<false, 2>(b, b, a); }
  u32 w[8]; f29_to_words(w, a); put(out, 0, g, w);
}
__global__ __launch_bounds__(256) void k_sqr32(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a, b; seed_fe(a, g, s); seed_fe(b, g, s + 1);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) { fe_sqr(a, a); fe_sqr(b, b); }
  fe_add(a, a, b); fe_normalize(a); put(out, 0, g, a.v);
}
__global__ __launch_bounds__(256) void k_sqr29(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  fe a0, b0; seed_fe(a0, g, s); seed_fe(b0, g, s + 1);
  fe29 a, b; f29_from_words(a, a0.v); f29_from_words(b, b0.v);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) { f29_sqr(a, a); f29_sqr(b, b); }
  f29_add(a, a, b);
  u32 w[8]; f29_to_words(w, a); put(out, 0, g, w);
}

// 3M + 4S doubling, same formula as gej_double (secp_group.cuh) with the
// magnitudes of the 9 x 29 layer: in/out X 1, Y 1, Z 2.
struct gej29 { fe29 x, y, z; };
__device__ __forceinline__ void gej29_double(gej29& r, const gej29& a) {
  fe29 A, B, C, D, E, t, u;
  f29_sqr(A, a.x);
  f29_sqr(B, a.y);
  f29_mul(t, a.y, a.z);              // 1 x 2
  f29_add(r.z, t, t);                // Z3 = 2YZ: mag 2
  f29_sqr(C, B);
  f29_mul(D, a.x, B);
  f29_mul3_norm(E, A);               // E = 3A: mag 1
  f29_sqr(t, E);                     // F
  f29_shl_norm<2>(D, D);             // 4D: mag 1
  f29_add(u, D, D);                  // 8D: mag 2
  f29_sub_norm<2>(r.x, t, u);        // X3 = F - 8D: mag 1
  f29_sub<1>(t, D, r.x);             // 4D - X3: mag 3
  f29_mul(t, E, t);                  // 1 x 3
  f29_shl_norm<3>(u, C);             // 8C: mag 1
  f29_sub_norm<1>(r.y, t, u);        // Y3 = E(4D - X3) - 8C: mag 1
}

__global__ __launch_bounds__(256) void k_dbl32(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  gej p; seed_fe(p.x, g, s); seed_fe(p.y, g, s + 1); seed_fe(p.z, g, s + 2);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) gej_double(p, p);
  fe_normalize(p.x); fe_normalize(p.y); fe_normalize(p.z);
  put(out, 0, g, p.x.v); put(out, 1, g, p.y.v); put(out, 2, g, p.z.v);
}
__global__ __launch_bounds__(256) void k_dbl29(u32* out, u32 s) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  fe x, y, z; seed_fe(x, g, s); seed_fe(y, g, s + 1); seed_fe(z, g, s + 2);
  gej29 p; f29_from_words(p.x, x.v); f29_from_words(p.y, y.v); f29_from_words(p.z, z.v);
#pragma unroll 1
  for (int i = 0; i < ITERS; ++i) gej29_double(p, p);
  u32 w[8];
  f29_to_words(w, p.x); put(out, 0, g, w);
  f29_to_words(w, p.y); put(out, 1, g, w);
  f29_to_words(w, p.z); put(out, 2, g, w);
}

typedef void (*kfn)(u32*, u32);
static int run(const char* name, kfn f, int blocks, u32* d, double ops_per_lane) {
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
  printf("{\"kernel\": \"%s\", \"ms\": %.3f, \"ops_per_s\": %.4e}\n", name, best, lanes * ops_per_lane / (best * 1e-3));
  return 0;
}
static int cmp(const char* what, u32* d0, u32* d1, size_t words) {
  u32* h0 = (u32*)malloc(words * 4); u32* h1 = (u32*)malloc(words * 4);
  CHK(hipMemcpy(h0, d0, words * 4, hipMemcpyDeviceToHost));
  CHK(hipMemcpy(h1, d1, words * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < words; ++i) bad += h0[i] != h1[i];
  printf("{\"check\": \"%s\", \"mismatched_words\": %zu, \"words\": %zu}\n", what, bad, words);
  free(h0); free(h1);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1) {   // latency mode: one wave per SIMD, ns per dependent operation
    const int blocks = 256;
    u32* d; CHK(hipMalloc(&d, (size_t)blocks * 256 * 24 * 4));
    printf("{\"mode\": \"latency, 1 wave/SIMD, ms for %d dependent ops per lane\"}\n", 2 * ITERS);
    if (run("lat fe_mul 8x32", k_mul32, blocks, d, 2.0 * ITERS)) return 1;
    if (run("lat fe_mul 9x29 one-chain", k_mul29, blocks, d, 2.0 * ITERS)) return 1;
    if (run("lat fe_mul 9x29 two-chain", k_mul29x2, blocks, d, 2.0 * ITERS)) return 1;
    if (run("lat fe_sqr 8x32", k_sqr32, blocks, d, 2.0 * ITERS)) return 1;
    if (run("lat fe_sqr 9x29", k_sqr29, blocks, d, 2.0 * ITERS)) return 1;
    if (run("lat gej_double 8x32", k_dbl32, blocks, d, ITERS)) return 1;
    if (run("lat gej_double 9x29", k_dbl29, blocks, d, ITERS)) return 1;
    return 0;
  }
  const int blocks = 256 * 8;
  const size_t lanes = (size_t)blocks * 256;
  u32 *d0, *d1;
  CHK(hipMalloc(&d0, lanes * 24 * 4)); CHK(hipMalloc(&d1, lanes * 24 * 4));
  if (run("fe_mul 8x32", k_mul32, blocks, d0, 2.0 * ITERS)) return 1;
  if (run("fe_mul 9x29", k_mul29, blocks, d1, 2.0 * ITERS)) return 1;
  if (cmp("mul", d0, d1, lanes * 8)) return 1;
  if (run("fe_mul 9x29 two-chain", k_mul29x2, blocks, d1, 2.0 * ITERS)) return 1;
  if (cmp("mul2", d0, d1, lanes * 8)) return 1;
  if (run("fe_sqr 8x32", k_sqr32, blocks, d0, 2.0 * ITERS)) return 1;
  if (run("fe_sqr 9x29", k_sqr29, blocks, d1, 2.0 * ITERS)) return 1;
  if (cmp("sqr", d0, d1, lanes * 8)) return 1;
  if (run("gej_double 8x32", k_dbl32, blocks, d0, ITERS)) return 1;
  if (run("gej_double 9x29", k_dbl29, blocks, d1, ITERS)) return 1;
  if (cmp("dbl", d0, d1, lanes * 24)) return 1;
  return 0;
}
