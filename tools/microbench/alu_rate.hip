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


// Generic: 8 independent 32-bit ops per iteration, "OP dst, src, dst" shapes.
#define K8_32(NAME, OPFMT)                                                             \
__global__ void NAME(uint64_t* out, uint32_t seed) {                                   \
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;                \
  uint32_t r0 = a, r1 = b, r2 = a ^ 1, r3 = b ^ 3, r4 = a + 7, r5 = b + 9, r6 = a * 3, r7 = b * 5; \
  for (int i = 0; i < ITERS; ++i) {                                                    \
    asm volatile(OPFMT(0) OPFMT(1) OPFMT(2) OPFMT(3) OPFMT(4) OPFMT(5) OPFMT(6) OPFMT(7) \
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(b), "v"(a)); \
  }                                                                                    \
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;  \
}
#define F_AND(k) "v_and_b32 %" #k ", %8, %" #k "\n\t"
#define F_ALIGN(k) "v_alignbit_b32 %" #k ", %8, %" #k ", 26\n\t"
#define F_LSHR(k) "v_lshrrev_b32 %" #k ", 26, %" #k "\n\t"
#define F_ADD3(k) "v_add3_u32 %" #k ", %8, %9, %" #k "\n\t"
#define F_MAD24(k) "v_mad_u32_u24 %" #k ", %8, %9, %" #k "\n\t"
#define F_MULLO(k) "v_mul_lo_u32 %" #k ", %8, %" #k "\n\t"
#define F_LSHLADD(k) "v_lshl_add_u32 %" #k ", %8, 3, %" #k "\n\t"
#define F_BFE(k) "v_bfe_u32 %" #k ", %" #k ", 3, 26\n\t"
K8_32(k_and, F_AND)
K8_32(k_align, F_ALIGN)
K8_32(k_lshr, F_LSHR)
K8_32(k_add3, F_ADD3)
K8_32(k_mad24, F_MAD24)
K8_32(k_mullo, F_MULLO)
K8_32(k_lshladd, F_LSHLADD)
K8_32(k_bfe, F_BFE)

// independent add-with-carry-out into distinct SGPR pairs (no VCC chain)
__global__ void k_addco_ind(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint32_t r0 = a, r1 = b, r2 = a ^ 1, r3 = b ^ 3, r4 = a + 7, r5 = b + 9, r6 = a * 3, r7 = b * 5;
  uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_add_co_u32 %0, %8, %12, %0\n\t" "v_add_co_u32 %1, %9, %12, %1\n\t"
      "v_add_co_u32 %2, %10, %12, %2\n\t" "v_add_co_u32 %3, %11, %12, %3\n\t"
      "v_add_co_u32 %4, %8, %12, %4\n\t" "v_add_co_u32 %5, %9, %12, %5\n\t"
      "v_add_co_u32 %6, %10, %12, %6\n\t" "v_add_co_u32 %7, %11, %12, %7\n\t"
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7),
        "+s"(c0), "+s"(c1), "+s"(c2), "+s"(c3) : "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7 ^ c0 ^ c1 ^ c2 ^ c3;
}

// 64-bit ops: v_lshrrev_b64 and v_lshl_add_u64 (gfx940+), 8 independent
__global__ void k_lshr64(uint64_t* out, uint32_t seed) {
  uint64_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761ull + seed;
  uint64_t r0 = a, r1 = b, r2 = a ^ 1, r3 = b ^ 3, r4 = a + 7, r5 = b + 9, r6 = a * 3, r7 = b * 5;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_lshrrev_b64 %0, 1, %0\n\t" "v_lshrrev_b64 %1, 1, %1\n\t" "v_lshrrev_b64 %2, 1, %2\n\t" "v_lshrrev_b64 %3, 1, %3\n\t"
      "v_lshrrev_b64 %4, 1, %4\n\t" "v_lshrrev_b64 %5, 1, %5\n\t" "v_lshrrev_b64 %6, 1, %6\n\t" "v_lshrrev_b64 %7, 1, %7\n\t"
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
}
__global__ void k_lshladd64(uint64_t* out, uint32_t seed) {
  uint64_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761ull + seed;
  uint64_t r0 = a, r1 = b, r2 = a ^ 1, r3 = b ^ 3, r4 = a + 7, r5 = b + 9, r6 = a * 3, r7 = b * 5;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_lshl_add_u64 %0, %8, 2, %0\n\t" "v_lshl_add_u64 %1, %8, 2, %1\n\t" "v_lshl_add_u64 %2, %8, 2, %2\n\t" "v_lshl_add_u64 %3, %8, 2, %3\n\t"
      "v_lshl_add_u64 %4, %8, 2, %4\n\t" "v_lshl_add_u64 %5, %8, 2, %5\n\t" "v_lshl_add_u64 %6, %8, 2, %6\n\t" "v_lshl_add_u64 %7, %8, 2, %7\n\t"
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
}
// mad chain with 4 waves/SIMD and ILP 4 (the field-mul regime), 32-bit x 32-bit + 64
__global__ void k_mad_ilp4(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint64_t r0 = a, r1 = b, r2 = a ^ 1, r3 = b ^ 3;
  uint64_t cc = 0;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_mad_u64_u32 %0, %4, %5, %6, %0\n\t" "v_mad_u64_u32 %1, %4, %5, %6, %1\n\t"
      "v_mad_u64_u32 %2, %4, %5, %6, %2\n\t" "v_mad_u64_u32 %3, %4, %5, %6, %3\n\t"
      "v_mad_u64_u32 %0, %4, %5, %6, %0\n\t" "v_mad_u64_u32 %1, %4, %5, %6, %1\n\t"
      "v_mad_u64_u32 %2, %4, %5, %6, %2\n\t" "v_mad_u64_u32 %3, %4, %5, %6, %3\n\t"
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+s"(cc) : "v"(a), "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ cc;
}

// Mixed streams: does a v_mov_b32 next to a 4-cycle op cost its own slot?
__global__ void k_mad_mov(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint64_t r0 = a, r1 = b, r2 = a ^ 1, r3 = b ^ 3;
  uint32_t m0 = a, m1 = b, m2 = a + 1, m3 = b + 1;
  uint64_t cc = 0;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_mad_u64_u32 %0, %8, %9, %10, %0\n\tv_mov_b32 %4, %9\n\t"
      "v_mad_u64_u32 %1, %8, %9, %10, %1\n\tv_mov_b32 %5, %10\n\t"
      "v_mad_u64_u32 %2, %8, %9, %10, %2\n\tv_mov_b32 %6, %9\n\t"
      "v_mad_u64_u32 %3, %8, %9, %10, %3\n\tv_mov_b32 %7, %10\n\t"
      "v_mad_u64_u32 %0, %8, %9, %10, %0\n\tv_mov_b32 %4, %10\n\t"
      "v_mad_u64_u32 %1, %8, %9, %10, %1\n\tv_mov_b32 %5, %9\n\t"
      "v_mad_u64_u32 %2, %8, %9, %10, %2\n\tv_mov_b32 %6, %10\n\t"
      "v_mad_u64_u32 %3, %8, %9, %10, %3\n\tv_mov_b32 %7, %9\n\t"
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3), "+s"(cc)
      : "v"(a), "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ cc ^ m0 ^ m1 ^ m2 ^ m3;
}
__global__ void k_addc_mov(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint32_t r0 = a, r1 = b, r2 = a ^ 1, r3 = b ^ 3, m0 = a, m1 = b, m2 = a + 1, m3 = b + 1;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_add_co_u32 %0, vcc, %8, %0\n\tv_mov_b32 %4, %8\n\t"
      "v_addc_co_u32 %1, vcc, %8, %1, vcc\n\tv_mov_b32 %5, %0\n\t"
      "v_addc_co_u32 %2, vcc, %8, %2, vcc\n\tv_mov_b32 %6, %1\n\t"
      "v_addc_co_u32 %3, vcc, %8, %3, vcc\n\tv_mov_b32 %7, %2\n\t"
      "v_addc_co_u32 %0, vcc, %8, %0, vcc\n\tv_mov_b32 %4, %3\n\t"
      "v_addc_co_u32 %1, vcc, %8, %1, vcc\n\tv_mov_b32 %5, %8\n\t"
      "v_addc_co_u32 %2, vcc, %8, %2, vcc\n\tv_mov_b32 %6, %8\n\t"
      "v_addc_co_u32 %3, vcc, %8, %3, vcc\n\tv_mov_b32 %7, %0\n\t"
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3) : "v"(b) : "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ m0 ^ m1 ^ m2 ^ m3;
}
__global__ void k_mov(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint32_t r0 = a, r1 = b, r2 = a ^ 1, r3 = b ^ 3, r4 = a + 7, r5 = b + 9, r6 = a * 3, r7 = b * 5;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
      "v_mov_b32 %0, %1\n\t" "v_mov_b32 %1, %2\n\t" "v_mov_b32 %2, %3\n\t" "v_mov_b32 %3, %4\n\t"
      "v_mov_b32 %4, %5\n\t" "v_mov_b32 %5, %6\n\t" "v_mov_b32 %6, %7\n\t" "v_mov_b32 %7, %8\n\t"
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
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
  if (run("v_and_b32", k_and, blocks, threads, d)) return 1;
  if (run("v_alignbit_b32", k_align, blocks, threads, d)) return 1;
  if (run("v_lshrrev_b32", k_lshr, blocks, threads, d)) return 1;
  if (run("v_add3_u32", k_add3, blocks, threads, d)) return 1;
  if (run("v_mad_u32_u24", k_mad24, blocks, threads, d)) return 1;
  if (run("v_mul_lo_u32", k_mullo, blocks, threads, d)) return 1;
  if (run("v_lshl_add_u32", k_lshladd, blocks, threads, d)) return 1;
  if (run("v_bfe_u32", k_bfe, blocks, threads, d)) return 1;
  if (run("v_add_co_u32 independent (sgpr carries)", k_addco_ind, blocks, threads, d)) return 1;
  if (run("v_lshrrev_b64", k_lshr64, blocks, threads, d)) return 1;
  if (run("v_lshl_add_u64", k_lshladd64, blocks, threads, d)) return 1;
  if (run("v_mad_u64_u32 ILP4 4w/SIMD", k_mad_ilp4, 256 * 4, threads, d)) return 1;
  if (run("v_mov_b32", k_mov, blocks, threads, d)) return 1;
  // pairs counted as 2 ops: a rate equal to the mad-only rate x2 means the mov is free
  if (run("mad+mov pairs (ops) 4w/SIMD", k_mad_mov, 256 * 4, threads, d, 16.0)) return 1;
  if (run("addc+mov pairs (ops) 4w/SIMD", k_addc_mov, 256 * 4, threads, d, 16.0)) return 1;
  if (run("v_addc_co_u32 chain 4w/SIMD", k_addc, 256 * 4, threads, d)) return 1;
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
