// isa_ops.hip -- one kernel per ladder operation of k_ecmult_k4, built from
// the product sources (gv_kernels.hip) with the exceptional-case branches of
// the mixed addition compiled out (GV_ISA_NOEXC), so each kernel body is the
// straight-line main path the ladder issues for that operation.
// tools/isa_ops.py compiles this to gfx950 assembly and counts instructions
// per kernel (minus the load/store frame measured by isa_frame).
#define GV_ISA_NOEXC 1
#include "../cosmos-sdk-rootchain_amd/csrc/gv_kernels.hip"

namespace gv {

GV_DEV void io_load(fe29& a, const u32* io, u32 C, u32 g, int k) {
#pragma unroll
  for (int i = 0; i < 9; ++i) a.n[i] = io[((size_t)k * 9 + i) * C + g];
}
GV_DEV void io_store(u32* io, u32 C, u32 g, int k, const fe29& a) {
#pragma unroll
  for (int i = 0; i < 9; ++i) io[((size_t)k * 9 + i) * C + g] = a.n[i];
}
GV_DEV void io_load_pt(gej29& a, const u32* io, u32 C, u32 g) {
  io_load(a.x, io, C, g, 0);
  io_load(a.y, io, C, g, 1);
  io_load(a.z, io, C, g, 2);
}
GV_DEV void io_store_pt(u32* io, u32 C, u32 g, const gej29& a) {
  io_store(io, C, g, 0, a.x);
  io_store(io, C, g, 1, a.y);
  io_store(io, C, g, 2, a.z);
}

// frame: load a point, store it back (subtracted from every count below)
__global__ __launch_bounds__(256) void isa_frame(u32* io, u32 C) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  gej29 a;
  io_load_pt(a, io, C, g);
  io_store_pt(io, C, g, a);
}

__global__ __launch_bounds__(256) void isa_mul(u32* io, u32 C) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  gej29 a;
  io_load_pt(a, io, C, g);
  f29x_mul(a.x, a.y, a.z);
  io_store_pt(io, C, g, a);
}

__global__ __launch_bounds__(256) void isa_sqr(u32* io, u32 C) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  gej29 a;
  io_load_pt(a, io, C, g);
  f29x_sqr(a.x, a.y);
  io_store_pt(io, C, g, a);
}

__global__ __launch_bounds__(256) void isa_dbl(u32* io, u32 C) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  gej29 a;
  io_load_pt(a, io, C, g);
  gej29x_double(a, a);
  io_store_pt(io, C, g, a);
}

// Q-table entry of the key arena, sign from the digit, mixed addition
__global__ __launch_bounds__(256) void isa_addq(u32* io, u32 C, const u32* kqt, const u32* qidx, const u32* dig) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  gej29 a;
  io_load_pt(a, io, C, g);
  bool inf = false;
  const int d = (int)(dig[g] << 16) >> 16;
  const u32 e = (u32)((d < 0 ? -d : d) - 1);
  fe29 x, y;
  load_qent29(x, y, kqt, qidx[g], e);
  if (d < 0) f29_neg<1>(y, y);
  gej29x_add_scaled(a, inf, x, y, a.z);
  io_store_pt(io, C, g, a);
}

// lambda*Q entry: the same plus the beta multiply
__global__ __launch_bounds__(256) void isa_addlq(u32* io, u32 C, const u32* kqt, const u32* qidx, const u32* dig) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  gej29 a;
  io_load_pt(a, io, C, g);
  bool inf = false;
  const int d = (int)dig[g] >> 16;
  const u32 e = (u32)((d < 0 ? -d : d) - 1);
  fe29 x, y;
  load_qent29(x, y, kqt, qidx[g], e);
  fe29 beta;
  f29_from_const(beta, kBeta);
  f29x_mul(x, x, beta);
  if (d < 0) f29_neg<1>(y, y);
  gej29x_add_scaled(a, inf, x, y, a.z);
  io_store_pt(io, C, g, a);
}

// G-table entry (8 x 32 words), lifted by the key table's Z
__global__ __launch_bounds__(256) void isa_addg(u32* io, u32 C, const u32* gtab, const u32* dig) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  gej29 a;
  io_load_pt(a, io, C, g);
  fe29 zq;
  io_load(zq, io, C, g, 3);
  bool inf = false;
  const int d = (int)dig[g];
  const u32 e = (u32)((d < 0 ? -d : d) - 1);
  fe29 x, y, az;
  load_gent29(x, y, gtab, e);
  if (d < 0) f29_neg<1>(y, y);
  f29x_mul(az, a.z, zq);
  gej29x_add_scaled(a, inf, x, y, az);
  io_store_pt(io, C, g, a);
}

// final check + ballot (stores only the bitmap: frame not subtracted)
__global__ __launch_bounds__(256) void isa_finish(u32* io, u32 C, const u32* flags, const u32* in_r, uint64_t* bits,
                                                  u32 n) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  gej29 a;
  io_load_pt(a, io, C, g);
  fe29 zq;
  io_load(zq, io, C, g, 3);
  ecmult_finish(a, false, zq, flags, in_r, bits, n, C, g);
}

}  // namespace gv
