// LayerNorm / GroupNorm over token-major (NHWC) fp16 activations, fp32 statistics (gfx950).
#include "vda_common.h"
#include "../../include/vda.h"

namespace {

// One wave per row; each lane owns up to 4 chunks of 8 channels (C <= 2048).
// Two-pass statistics from registers: mean, then mean of squared deviations (as torch does).
__global__ __launch_bounds__(256) void layernorm_kernel(const h16* __restrict__ x, long ldx,
                                                        h16* __restrict__ y, const float* __restrict__ g,
                                                        const float* __restrict__ b, int rows, int C,
                                                        float eps, int skip_period) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const long src_row = skip_period > 0 ? (long)row + row / skip_period + 1 : (long)row;
  const h16* xr = x + src_row * ldx;
  const int nch = C >> 3;
  float v[4][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      h8 t = __builtin_bit_cast(h8, ldg16(xr + c * 8));
#pragma unroll
      for (int j = 0; j < 8; ++j) { v[i][j] = (float)t[j]; s += v[i][j]; }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { float d = v[i][j] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)C + eps);
  h16* yr = y + (long)row * C;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      const f4 g0 = *reinterpret_cast<const f4*>(g + c * 8), g1 = *reinterpret_cast<const f4*>(g + c * 8 + 4);
      const f4 b0 = *reinterpret_cast<const f4*>(b + c * 8), b1 = *reinterpret_cast<const f4*>(b + c * 8 + 4);
      h8 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = (h16)((v[i][j] - mean) * rstd * g0[j] + b0[j]);
        o[j + 4] = (h16)((v[i][j + 4] - mean) * rstd * g1[j] + b1[j]);
      }
      stg16(yr + c * 8, __builtin_bit_cast(uint4, o));
    }
  }
}

// GroupNorm: one block per (frame, group).  Pass 1: mean; pass 2: centred second moment;
// pass 3: normalise + affine.  Slab = S rows x cg contiguous channels at row stride C.
// Loads are VW halfs wide (VW = 8/4/2 chosen from cg).
template <int VW>
__global__ __launch_bounds__(256) void groupnorm_kernel(const h16* __restrict__ x, h16* __restrict__ y,
                                                        const float* __restrict__ gam, const float* __restrict__ bet,
                                                        int S, int C, int groups, float eps) {
  typedef _Float16 hv __attribute__((ext_vector_type(VW)));
  const int f = blockIdx.x / groups, grp = blockIdx.x % groups;
  const int cg = C / groups;
  const int vpr = cg / VW;  // vectors per row
  const long nvec = (long)S * vpr;
  const h16* base = x + (long)f * S * C + grp * cg;
  h16* obase = y + (long)f * S * C + grp * cg;
  __shared__ float red[4];
  auto block_sum = [&](float v) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float t = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    return t;
  };
  float s = 0.f;
  for (long i = threadIdx.x; i < nvec; i += 256) {
    const long r = i / vpr; const int c = (int)(i - r * vpr) * VW;
    hv t = *reinterpret_cast<const hv*>(base + r * C + c);
#pragma unroll
    for (int j = 0; j < VW; ++j) s += (float)t[j];
  }
  const float cnt = (float)S * (float)cg;
  const float mean = block_sum(s) / cnt;
  float q = 0.f;
  for (long i = threadIdx.x; i < nvec; i += 256) {
    const long r = i / vpr; const int c = (int)(i - r * vpr) * VW;
    hv t = *reinterpret_cast<const hv*>(base + r * C + c);
#pragma unroll
    for (int j = 0; j < VW; ++j) { float d = (float)t[j] - mean; q += d * d; }
  }
  const float rstd = rsqrtf(block_sum(q) / cnt + eps);
  for (long i = threadIdx.x; i < nvec; i += 256) {
    const long r = i / vpr; const int c = (int)(i - r * vpr) * VW;
    hv t = *reinterpret_cast<const hv*>(base + r * C + c);
    hv o;
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const int ch = grp * cg + c + j;
      o[j] = (h16)(((float)t[j] - mean) * rstd * gam[ch] + bet[ch]);
    }
    *reinterpret_cast<hv*>(obase + r * C + c) = o;
  }
}

}  // namespace

extern "C" int vda_layernorm(const void* x, int64_t ldx, void* y, const float* gamma, const float* beta,
                             int32_t rows, int32_t C, float eps, int32_t skip_period, void* stream) {
  VDA_CHECK_ARG(x && y && gamma && beta, "null pointer");
  VDA_CHECK_ARG(rows > 0 && C > 0 && C % 8 == 0 && C <= 2048, "C must be a multiple of 8, <= 2048");
  VDA_CHECK_ARG(ldx % 8 == 0 && ldx >= C, "ldx must be a multiple of 8 and >= C");
  VDA_CHECK_ARG(skip_period >= 0, "skip_period >= 0");
  hipLaunchKernelGGL(layernorm_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     (const h16*)x, (long)ldx, (h16*)y, gamma, beta, rows, C, eps, skip_period);
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_groupnorm(const void* x, void* y, const float* gamma, const float* beta, int32_t F,
                             int32_t S, int32_t C, int32_t groups, float eps, float* ws, void* stream) {
  (void)ws;
  VDA_CHECK_ARG(x && y && gamma && beta, "null pointer");
  VDA_CHECK_ARG(F > 0 && S > 0 && groups > 0 && C % groups == 0, "C must be divisible by groups");
  const int cg = C / groups;
  VDA_CHECK_ARG(cg % 2 == 0, "channels per group must be even");
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(F * groups);
  if (cg % 8 == 0)
    hipLaunchKernelGGL(groupnorm_kernel<8>, grid, dim3(256), 0, st, (const h16*)x, (h16*)y, gamma, beta, S, C, groups, eps);
  else if (cg % 4 == 0)
    hipLaunchKernelGGL(groupnorm_kernel<4>, grid, dim3(256), 0, st, (const h16*)x, (h16*)y, gamma, beta, S, C, groups, eps);
  else
    hipLaunchKernelGGL(groupnorm_kernel<2>, grid, dim3(256), 0, st, (const h16*)x, (h16*)y, gamma, beta, S, C, groups, eps);
  VDA_LAUNCH_CHECK();
  return 0;
}
