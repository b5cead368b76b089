// Integer-ALU issue-rate microbenchmark for gfx950 (MI355X).
// Measures per-chip throughput of the instructions the secp256k1 field
// arithmetic is built from, so bench.py's roofline denominator (P_mul) is a
// measured number rather than a datasheet guess (SURVEY.md §8d "Peak denominator").
//   v_mad_u64_u32  : 32x32->64 multiply + 64-bit add (one "product")
//   v_mul_hi_u32   : high half of 32x32
//   v_addc_co_u32  : add with carry (full-rate reference)
//   v_fma_f64      : fp64 FMA (alternative radix-2^52 arithmetic)
// Each lane runs 8 independent chains (ILP 8) for ITERS iterations; a grid of
// many waves per SIMD hides latency.  Result: instructions/s chip-wide.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_mad(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint64_t r0 = a, r1 = b, r2 = a ^ 1, r3 = b ^ 3, r4 = a + 7, r5 = b + 9, r6 = a * 3, r7 = b * 5;
  uint64_t cc = 0;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_mad_u64_u32 %0, %8, %9, %10, %0\n\t"
      "v_mad_u64_u32 %1, %8, %9, %10, %1\n\t"
      "v_mad_u64_u32 %2, %8, %9, %10, %2\n\t"
      "v_mad_u64_u32 %3, %8, %9, %10, %3\n\t"
      "v_mad_u64_u32 %4, %8, %9, %10, %4\n\t"
      "v_mad_u64_u32 %5, %8, %9, %10, %5\n\t"
      "v_mad_u64_u32 %6, %8, %9, %10, %6\n\t"
      "v_mad_u64_u32 %7, %8, %9, %10, %7\n\t"
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7), "+s"(cc)
      : "v"(a), "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7 ^ cc;
}

__global__ void k_mulhi(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint32_t r0 = a, r1 = b, r2 = a ^ 1, r3 = b ^ 3, r4 = a + 7, r5 = b + 9, r6 = a * 3, r7 = b * 5;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_mul_hi_u32 %0, %8, %0\n\t"
      "v_mul_hi_u32 %1, %8, %1\n\t"
      "v_mul_hi_u32 %2, %8, %2\n\t"
      "v_mul_hi_u32 %3, %8, %3\n\t"
      "v_mul_hi_u32 %4, %8, %4\n\t"
      "v_mul_hi_u32 %5, %8, %5\n\t"
      "v_mul_hi_u32 %6, %8, %6\n\t"
      "v_mul_hi_u32 %7, %8, %7\n\t"
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
      : "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
}

__global__ void k_addc(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint32_t r0 = a, r1 = b, r2 = a ^ 1, r3 = b ^ 3, r4 = a + 7, r5 = b + 9, r6 = a * 3, r7 = b * 5;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_add_co_u32 %0, vcc, %8, %0\n\t"
      "v_addc_co_u32 %1, vcc, %8, %1, vcc\n\t"
      "v_addc_co_u32 %2, vcc, %8, %2, vcc\n\t"
      "v_addc_co_u32 %3, vcc, %8, %3, vcc\n\t"
      "v_addc_co_u32 %4, vcc, %8, %4, vcc\n\t"
      "v_addc_co_u32 %5, vcc, %8, %5, vcc\n\t"
      "v_addc_co_u32 %6, vcc, %8, %6, vcc\n\t"
      "v_addc_co_u32 %7, vcc, %8, %7, vcc\n\t"
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
      : "v"(b) : "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
}

__global__ void k_fma64(uint64_t* out, uint32_t seed) {
  double a = 1.0000001 + threadIdx.x * 1e-9, b = 0.999999 + seed * 1e-12;
  double r0 = a, r1 = b, r2 = a + 1, r3 = b + 1, r4 = a + 2, r5 = b + 2, r6 = a + 3, r7 = b + 3;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_fma_f64 %0, %8, %0, %9\n\t"
      "v_fma_f64 %1, %8, %1, %9\n\t"
      "v_fma_f64 %2, %8, %2, %9\n\t"
      "v_fma_f64 %3, %8, %3, %9\n\t"
      "v_fma_f64 %4, %8, %4, %9\n\t"
      "v_fma_f64 %5, %8, %5, %9\n\t"
      "v_fma_f64 %6, %8, %6, %9\n\t"
      "v_fma_f64 %7, %8, %7, %9\n\t"
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
      : "v"(b), "v"(a));
  }
  double s = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
  out[blockIdx.x * blockDim.x + threadIdx.x] = __double_as_longlong(s);
}


// Dependent chain: every mad consumes the previous result (ILP 1).
__global__ void k_mad_dep(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint64_t r0 = a;
  uint64_t cc = 0;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
      "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
      "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
      "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
      "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
      "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
      "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
      "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
      : "+v"(r0), "+s"(cc) : "v"(a), "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ cc;
}

// mad + addc pair chain (the product-scanning inner step), ILP 1.
__global__ void k_madc_dep(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint64_t r0 = a; uint32_t w = 0;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc\n\t"
      : "+v"(r0), "+v"(w) : "v"(a), "v"(b) : "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ w;
}

// Independent 32-bit adds (no carry chain): the full-rate VALU reference.
__global__ void k_add(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint32_t r0 = a, r1 = b, r2 = a ^ 1, r3 = b ^ 3, r4 = a + 7, r5 = b + 9, r6 = a * 3, r7 = b * 5;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_add_u32 %0, %8, %0\n\t" "v_add_u32 %1, %8, %1\n\t" "v_add_u32 %2, %8, %2\n\t" "v_add_u32 %3, %8, %3\n\t"
      "v_add_u32 %4, %8, %4\n\t" "v_add_u32 %5, %8, %5\n\t" "v_add_u32 %6, %8, %6\n\t" "v_add_u32 %7, %8, %7\n\t"
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
}

// Effective shader clock under an integer-VALU load: s_memtime ticks at the
// shader clock, s_memrealtime at a constant 100 MHz.
__global__ void k_clock(uint64_t* out, uint32_t seed) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint64_t x0 = a, x1 = b, x2 = a ^ 5, x3 = b ^ 9;
  for (int i = 0; i < ITERS * 4; ++i) {
    asm volatile("v_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_mad_u64_u32 %1, vcc, %4, %5, %1\n\t"
                 "v_mad_u64_u32 %2, vcc, %4, %5, %2\n\tv_mad_u64_u32 %3, vcc, %4, %5, %3"
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(a), "v"(b) : "vcc");
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = t1 - t0; out[2 * blockIdx.x + 1] = r1 - r0; }
  if ((x0 ^ x1 ^ x2 ^ x3) == 0x123456789ull) out[0] = 0;
}

typedef void (*kfn)(uint64_t*, uint32_t);

static int run(const char* name, kfn f, int blocks, int threads, uint64_t* d, double per_iter = 8.0) {
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 1u);  // warm
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)rep);
    CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
  }
  double insts = (double)blocks * threads * ITERS * per_iter;
  double rate = insts / (best * 1e-3);
  // per CU per clock at 2.4 GHz nominal, 256 CUs
  printf("{\"inst\": \"%s\", \"lane_ops_per_s\": %.4e, \"lane_ops_per_clk_per_cu_at_2p4GHz\": %.2f, \"ms\": %.3f}\n",
         name, rate, rate / (256.0 * 2.4e9), best);
  return 0;
}

int main() {
  int blocks = 256 * 16, threads = 256;
  uint64_t* d; CHK(hipMalloc(&d, (size_t)blocks * threads * 8));
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  if (run("v_mad_u64_u32", k_mad, blocks, threads, d)) return 1;
  if (run("v_mul_hi_u32", k_mulhi, blocks, threads, d)) return 1;
  if (run("v_addc_co_u32", k_addc, blocks, threads, d)) return 1;
  if (run("v_fma_f64", k_fma64, blocks, threads, d)) return 1;
  if (run("v_add_u32", k_add, blocks, threads, d)) return 1;
  // dependent chains at 8 waves/SIMD (16 blocks/CU of 256) and at 2 waves/SIMD
  if (run("v_mad_u64_u32 dep-chain 8w/SIMD", k_mad_dep, blocks, threads, d)) return 1;
  if (run("v_mad_u64_u32 dep-chain 2w/SIMD", k_mad_dep, 256 * 2, threads, d)) return 1;
  if (run("mad+addc dep-pair 8w/SIMD (products)", k_madc_dep, blocks, threads, d, 4.0)) return 1;
  if (run("mad+addc dep-pair 2w/SIMD (products)", k_madc_dep, 256 * 2, threads, d, 4.0)) return 1;
  if (run("v_mad_u64_u32 ILP8 2w/SIMD", k_mad, 256 * 2, threads, d)) return 1;
  {
    int nb = 256 * 8;
    hipLaunchKernelGGL(k_clock, dim3(nb), dim3(256), 0, 0, d, 3u);
    CHK(hipDeviceSynchronize());
    uint64_t* h = (uint64_t*)malloc(16 * nb);
    CHK(hipMemcpy(h, d, 16 * nb, hipMemcpyDeviceToHost));
    double tk = 0, rt = 0;
    for (int i = 0; i < nb; ++i) { tk += h[2 * i]; rt += h[2 * i + 1]; }
    printf("{\"effective_shader_clock_GHz\": %.3f}\n", tk / rt * 0.1);
    free(h);
  }
  CHK(hipFree(d));
  return 0;
}
