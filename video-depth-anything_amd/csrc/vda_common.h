// Shared device helpers for libvda (gfx950 / CDNA4 only).
//
// Every hot op of the Video-Depth-Anything clip forward runs through
// kernels built on these types.  Activations and weights are fp16 in HBM, accumulation and
// all normalisation / softmax statistics are fp32.  Activations are token-major (NHWC) end
// to end, so the reference's permute/rearrange calls become index math in the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "vda_tune.h"

typedef _Float16 h16;
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f16x __attribute__((ext_vector_type(16)));

#define VDA_LDS __attribute__((address_space(3)))

__device__ __forceinline__ f4 mfma16(h8 a, h8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f16x mfma32(h8 a, h8 b, f16x c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// Hardware-transposed LDS read (ds_read_b64_tr_b16): per 16-lane group, lane 4q+p supplies the
// address of row q / columns 4p..4p+3 of a 4x16 block; lane i receives column i (4 rows).
__device__ __forceinline__ h4 lds_read_tr16(const h16* p) {
  s4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VDA_LDS s4*)(p));
  return __builtin_bit_cast(h4, t);
}

// Exact-erf GELU (nn.GELU default, not the tanh form).  erf by Abramowitz & Stegun 7.1.26
// (|error| <= 1.5e-7, far below fp16 output rounding): one v_rcp, one v_exp, five FMAs - about a
// third of the instructions of the library erff, which matters in the GEMM epilogues.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * ax);
  float y = 1.061405429f;
  y = fmaf(y, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  y *= t;
  const float e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  const float r = fmaf(-y, e, 1.0f);
  return copysignf(r, x);
}
// Bilinear blend of 8 fp16 channels in fp32, rounded to fp16: (1-wy)*((1-wx)*a + wx*b) + wy*((1-wx)*c + wx*d)
// with every product / fma spelled out, so the resize kernel and the depth head's fused patch builder
// produce bit-identical values (no compiler contraction choices in between).
// Bilinear (align_corners=True) blend weight of output coordinate o at source scale sc, source index
// i0 = (int)(sc * o): the exact product minus i0 in one fma.  Spelled out so that every resize site
// (upsample kernel, the fused-resize convs, the res2 gather, the implicit-GEMM loader) forms the same
// bits whatever the compiler's contraction choice in its code shape (a restructured loop could keep the
// rounded product instead and move w by an ulp: DESIGN.md §3, round-4 levers).
__device__ __forceinline__ float ac_weight(float sc, float o, int i0) { return __builtin_fmaf(sc, o, -(float)i0); }

__device__ __forceinline__ h8 bilerp8(h8 a, h8 b, h8 c, h8 d, float wx, float wy) {
  const float ux = 1.f - wx, uy = 1.f - wy;
  h8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float top = __builtin_fmaf(wx, (float)b[j], ux * (float)a[j]);
    const float bot = __builtin_fmaf(wx, (float)d[j], ux * (float)c[j]);
    o[j] = (h16)__builtin_fmaf(wy, bot, uy * top);
  }
  return o;
}
// The same blend with v_fma_mix_f32 reading the fp16 channels straight out of the packed registers
// (exact f16 -> f32 in the FMA, one rounding): bit-identical to bilerp8 (ux * a as fma(ux, a, -0) keeps
// the product's sign of zero) in 6 VALU per channel instead of 10 (4 conversions + 6 ops, which
// -O3 also SLP-packs into v_pk_*_f32, slow beside MFMAs).
__device__ __forceinline__ float fma_mix_lo(float a, unsigned hb, float c) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(d) : "v"(a), "v"(hb), "v"(c));
  return d;
}
__device__ __forceinline__ float fma_mix_hi(float a, unsigned hb, float c) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(d) : "v"(a), "v"(hb), "v"(c));
  return d;
}
__device__ __forceinline__ float mul_f32(float a, float b) {  // single v_mul_f32 (no SLP packing)
  float d;
  asm("v_mul_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ float fma_f32(float a, float b, float c) {
  float d;
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ uint4 bilerp8_mix(uint4 a, uint4 b, uint4 c, uint4 d, float wx, float wy) {
  const float ux = 1.f - wx, uy = 1.f - wy;
  const unsigned A[4] = {a.x, a.y, a.z, a.w}, B[4] = {b.x, b.y, b.z, b.w};
  const unsigned Cc[4] = {c.x, c.y, c.z, c.w}, D[4] = {d.x, d.y, d.z, d.w};
  unsigned o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float tl = fma_mix_lo(wx, B[j], fma_mix_lo(ux, A[j], -0.f));
    const float th = fma_mix_hi(wx, B[j], fma_mix_hi(ux, A[j], -0.f));
    const float bl = fma_mix_lo(wx, D[j], fma_mix_lo(ux, Cc[j], -0.f));
    const float bh = fma_mix_hi(wx, D[j], fma_mix_hi(ux, Cc[j], -0.f));
    const float ol = fma_f32(wy, bl, mul_f32(uy, tl));
    const float oh = fma_f32(wy, bh, mul_f32(uy, th));
    typedef float f2v __attribute__((ext_vector_type(2)));
    o[j] = __builtin_bit_cast(unsigned, __builtin_convertvector(f2v{ol, oh}, h2));
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Exchange with the partner lane across 16-lane rows (lane ^ 16) resp. wave halves (lane ^ 32):
// v_permlane16/32_swap with both operands holding v leaves {own, partner} in the pair.  Inline asm
// because the ROCm 7.2 builtins miscompile exactly this case: with the same value for both operands
// the second result is read from the first's register (the fmax / add of the pair folds to one
// value).  s_nop 1 = the 2 wait states a VALU write needs before the swap reads it.
__device__ __forceinline__ void swap16_pair(float v, float& a, float& b) {
  a = v; b = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void swap32_pair(float v, float& a, float& b) {
  a = v; b = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ float half_max(float v) { float a, b; swap32_pair(v, a, b); return fmaxf(a, b); }
__device__ __forceinline__ float half_sum(float v) { float a, b; swap32_pair(v, a, b); return a + b; }
// max over the 4 lane groups of 16 (lane bits 4 and 5) with VALU permlane swaps, no LDS traffic
__device__ __forceinline__ float group_max4(float v) {
  float a, b;
  swap16_pair(v, a, b);
  return half_max(fmaxf(a, b));
}

__device__ __forceinline__ uint4 ldg16(const void* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ void stg16(void* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }

// ReLU on fp16 bit patterns: a negative half is a negative int16, so max_i16(x, 0) is relu(x)
// (-0 and negative NaNs -> +0).  Packed: one v_pk_max_i16 per two values, no SLP pass needed.
typedef short s8v __attribute__((ext_vector_type(8)));
__device__ __forceinline__ h8 relu8(h8 x) {
  return __builtin_bit_cast(h8, __builtin_elementwise_max(__builtin_bit_cast(s8v, x), s8v{0, 0, 0, 0, 0, 0, 0, 0}));
}
__device__ __forceinline__ uint4 relu_h8(uint4 v) { return __builtin_bit_cast(uint4, relu8(__builtin_bit_cast(h8, v))); }

// Compute units of the current device (hipDeviceAttributeMultiprocessorCount), memoised per device:
// a read-only device property, not tuning state (vda_misc.hip).
int vda_cu_count();

// Error reporting across the C ABI (never throws).
int vda_set_error(int code, const char* msg);
#define VDA_CHECK_ARG(cond, msg) \
  do { if (!(cond)) return vda_set_error(-22, msg); } while (0)
#define VDA_LAUNCH_CHECK() \
  do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return vda_set_error((int)_e, hipGetErrorString(_e)); } while (0)
