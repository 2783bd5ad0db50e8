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

// Row statistics only (the LN-folded GEMM, vda_epilogue.ln_stats): the same two-pass mean / rstd as
// layernorm_kernel, one wave per row, written as float2.  Reads the row once, writes 8 bytes.
__global__ __launch_bounds__(256) void row_stats_kernel(const h16* __restrict__ x, long ldx, float2* __restrict__ st,
                                                        int rows, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const h16* xr = x + (long)row * ldx;
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
  if (lane == 0) st[row] = make_float2(mean, rstd);
}

// Per-row partial (sum, sum of squares) over 256-column blocks of an fp16 matrix: the fallback for
// vda_epilogue.stats_out when the producing GEMM did not take the phased kernel (which computes them
// in its epilogue).  One wave per (row, block): 32 lanes x 8 columns.
__global__ __launch_bounds__(256) void row_partials_kernel(const h16* __restrict__ y, long ldy, float2* __restrict__ st,
                                                           int rows, int N, int P) {
  const int lane = threadIdx.x & 63;
  const long item = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= (long)rows * P) return;
  const int row = (int)(item / P), blk = (int)(item - (long)row * P);
  const int c = blk * 256 + (lane & 31) * 8;
  float s = 0.f, q = 0.f;
  if (lane < 32 && c < N) {
    const h8 t = __builtin_bit_cast(h8, ldg16(y + (long)row * ldy + c));
#pragma unroll
    for (int j = 0; j < 8; ++j) { const float v = (float)t[j]; s += v; q = fmaf(v, v, q); }
  }
  s = wave_sum(s);
  q = wave_sum(q);
  if (lane == 0) st[item] = make_float2(s, q);
}

// Narrow rows (C <= 512, the motion modules' C = 256 / 128): one wave would leave lanes idle and
// wait on one 512-B row, so LPR = C / 8 lanes own a row (one 16-B chunk each) and a wave normalises
// 64 / LPR rows; the same two-pass statistics, reduced over the row's LPR lanes only.
template <int LPR>
__global__ __launch_bounds__(256) void layernorm_narrow_kernel(const h16* __restrict__ x, long ldx,
                                                               h16* __restrict__ y, const float* __restrict__ g,
                                                               const float* __restrict__ b, int rows, int C,
                                                               float eps, int skip_period) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane / LPR, c = lane % LPR;
  const int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + sub;
  const bool ok = row < rows;
  const int r = ok ? row : rows - 1;  // every lane joins the shuffles
  const long src_row = skip_period > 0 ? (long)r + r / skip_period + 1 : (long)r;
  const h8 t = __builtin_bit_cast(h8, ldg16(x + src_row * ldx + c * 8));
  float v[8], s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { v[j] = (float)t[j]; s += v[j]; }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / (float)C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { const float d = v[j] - mean; q += d * d; }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rstd = rsqrtf(q / (float)C + eps);
  const f4 g0 = *reinterpret_cast<const f4*>(g + c * 8), g1 = *reinterpret_cast<const f4*>(g + c * 8 + 4);
  const f4 b0 = *reinterpret_cast<const f4*>(b + c * 8), b1 = *reinterpret_cast<const f4*>(b + c * 8 + 4);
  h8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = (h16)((v[j] - mean) * rstd * g0[j] + b0[j]);
    o[j + 4] = (h16)((v[j + 4] - mean) * rstd * g1[j] + b1[j]);
  }
  if (ok) stg16(y + (long)row * C + c * 8, __builtin_bit_cast(uint4, o));
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

// GroupNorm, three coalesced passes over [F, S, C] (used when the caller passes a workspace):
//   gn_partial:  block (frame, chunk of gn_rows(C) rows) reads whole rows (16 B per thread) and writes
//                per-channel partial sums of d and d^2, d = x - shift_g (shift_g = the group's first
//                value of the frame, so the one-pass variance does not cancel);
//   gn_finalize: per (frame, group) mean and rstd from the partials, fixed summation order;
//   gn_apply:    y = (x - mean) * rstd * gamma + beta, same row-chunk grid.
// Deterministic (no atomics).  The per-(frame, group) kernel above reads strided 16-B slivers of
// every row three times; these read each row once per pass with full-row coalescing.
// Rows per (frame, chunk) block: 128, or 32 for C >= 512 (there 128 rows are 64 sequential loads per
// thread and a 19^2 map gave 96 blocks for 256 CUs: 34.7 us for 24 MB, round 4's forward trace)
__host__ __device__ constexpr int gn_rows(int C) { return C >= 512 ? 32 : 128; }

__device__ __forceinline__ void gn_layout(int C, int& cpr, int& rpi) {
  cpr = C >> 3;          // 8-channel chunks per row
  rpi = 256 / cpr;       // rows per block iteration
}

__global__ __launch_bounds__(256) void gn_partial_kernel(const h16* __restrict__ x, float* __restrict__ part, int S, int C,
                                                         int groups, int nchunk) {
  __shared__ float red[256 * 16];  // [thread][sum d x8 | sum d^2 x8] (16 KB)
  const int f = blockIdx.x / nchunk, ch = blockIdx.x % nchunk;
  int cpr, rpi;
  gn_layout(C, cpr, rpi);
  const int tid = threadIdx.x;
  const int cc = tid % cpr, r0 = tid / cpr;
  const int cg = C / groups;
  const h16* fx = x + (long)f * S * C;
  float sh[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sh[j] = (float)fx[((cc * 8 + j) / cg) * cg];
    s1[j] = 0.f;
    s2[j] = 0.f;
  }
  if (r0 < rpi) {
    const int rend = min(S, (ch + 1) * gn_rows(C));
#pragma unroll 4
    for (int r = ch * gn_rows(C) + r0; r < rend; r += rpi) {
      const h8 v = __builtin_bit_cast(h8, ldg16(fx + (long)r * C + cc * 8));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = (float)v[j] - sh[j];
        s1[j] += d;
        s2[j] = fmaf(d, d, s2[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[tid * 16 + j] = s1[j];
    red[tid * 16 + 8 + j] = s2[j];
  }
  __syncthreads();
  if (tid < cpr) {  // fold the rpi row-lanes of chunk column tid, fixed order
    float a1[8], a2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a1[j] = 0.f; a2[j] = 0.f; }
    for (int q = 0; q < rpi; ++q) {
      const float* rr = &red[(q * cpr + tid) * 16];
#pragma unroll
      for (int j = 0; j < 8; ++j) { a1[j] += rr[j]; a2[j] += rr[8 + j]; }
    }
    float* out = part + ((long)(f * nchunk + ch) * C + tid * 8) * 2;
#pragma unroll
    for (int j = 0; j < 8; ++j) { out[2 * j] = a1[j]; out[2 * j + 1] = a2[j]; }
  }
}

__global__ __launch_bounds__(64) void gn_finalize_kernel(const h16* __restrict__ x, const float* __restrict__ part,
                                                         float* __restrict__ stats, int S, int C, int groups, int nchunk,
                                                         float eps) {
  const int f = blockIdx.x / groups, g = blockIdx.x % groups;
  const int cg = C / groups;
  const int lane = threadIdx.x;
  float a1 = 0.f, a2 = 0.f;
  const int n = nchunk * cg;
#pragma unroll 8  // loads in flight; the sums keep their order
  for (int i = lane; i < n; i += 64) {
    const int chn = i / cg, c = g * cg + (i - chn * cg);
    const float* p = part + ((long)(f * nchunk + chn) * C + c) * 2;
    a1 += p[0];
    a2 += p[1];
  }
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  if (lane == 0) {
    const float cnt = (float)S * (float)cg;
    const float md = a1 / cnt;
    const float var = fmaxf(a2 / cnt - md * md, 0.f);
    stats[(f * groups + g) * 2] = (float)x[(long)f * S * C + g * cg] + md;
    stats[(f * groups + g) * 2 + 1] = rsqrtf(var + eps);
  }
}

__global__ __launch_bounds__(256) void gn_apply_kernel(const h16* __restrict__ x, h16* __restrict__ y,
                                                       const float* __restrict__ stats, const float* __restrict__ gam,
                                                       const float* __restrict__ bet, int S, int C, int groups, int nchunk) {
  const int f = blockIdx.x / nchunk, ch = blockIdx.x % nchunk;
  int cpr, rpi;
  gn_layout(C, cpr, rpi);
  const int tid = threadIdx.x;
  const int cc = tid % cpr, r0 = tid / cpr;
  if (r0 >= rpi) return;
  const int cg = C / groups;
  float sc[8], of[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cc * 8 + j, g = c / cg;
    const float mean = stats[(f * groups + g) * 2], rstd = stats[(f * groups + g) * 2 + 1];
    sc[j] = rstd * gam[c];
    of[j] = bet[c] - mean * sc[j];
  }
  const long fo = (long)f * S * C;
  const int rend = min(S, (ch + 1) * gn_rows(C));
#pragma unroll 4
  for (int r = ch * gn_rows(C) + r0; r < rend; r += rpi) {
    const h8 v = __builtin_bit_cast(h8, ldg16(x + fo + (long)r * C + cc * 8));
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (h16)fmaf((float)v[j], sc[j], of[j]);
    stg16(y + fo + (long)r * C + cc * 8, __builtin_bit_cast(uint4, o));
  }
}

}  // namespace

extern "C" int vda_row_stats(const void* x, int64_t ldx, float* stats, int32_t rows, int32_t C, float eps,
                             void* stream) {
  VDA_CHECK_ARG(x && stats, "null pointer");
  VDA_CHECK_ARG(rows > 0 && C > 0 && C % 8 == 0 && C <= 2048, "C must be a multiple of 8, <= 2048");
  VDA_CHECK_ARG(ldx % 8 == 0 && ldx >= C, "ldx must be a multiple of 8 and >= C");
  hipLaunchKernelGGL(row_stats_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, (const h16*)x, (long)ldx,
                     (float2*)stats, rows, C, eps);
  VDA_LAUNCH_CHECK();
  return 0;
}

int vda_row_partials_launch(const void* y, int64_t ldy, float* out, int32_t rows, int32_t N, hipStream_t stream) {
  // the kernel reads whole 16-byte pieces of y
  VDA_CHECK_ARG(N % 8 == 0 && ldy % 8 == 0 && (uintptr_t)y % 16 == 0,
                "stats_out: the output needs N % 8 == 0, ldy % 8 == 0 and 16-byte alignment");
  const int P = (N + 255) / 256;
  const long items = (long)rows * P;
  hipLaunchKernelGGL(row_partials_kernel, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, stream,
                     (const h16*)y, (long)ldy, (float2*)out, rows, N, P);
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_layernorm(const void* x, int64_t ldx, void* y, const float* gamma, const float* beta,
                             int32_t rows, int32_t C, float eps, int32_t skip_period, void* stream) {
  VDA_CHECK_ARG(x && y && gamma && beta, "null pointer");
  VDA_CHECK_ARG(rows > 0 && C > 0 && C % 8 == 0 && C <= 2048, "C must be a multiple of 8, <= 2048");
  VDA_CHECK_ARG(ldx % 8 == 0 && ldx >= C, "ldx must be a multiple of 8 and >= C");
  VDA_CHECK_ARG(skip_period >= 0, "skip_period >= 0");
  hipStream_t st = (hipStream_t)stream;
  if (C == 256 || C == 512 || C == 128) {
    const int lpr = C / 8, rpb = 4 * (64 / lpr);  // rows per 256-thread block
    const dim3 grid((rows + rpb - 1) / rpb);
    if (lpr == 16)
      hipLaunchKernelGGL(layernorm_narrow_kernel<16>, grid, dim3(256), 0, st, (const h16*)x, (long)ldx, (h16*)y, gamma,
                         beta, rows, C, eps, skip_period);
    else if (lpr == 32)
      hipLaunchKernelGGL(layernorm_narrow_kernel<32>, grid, dim3(256), 0, st, (const h16*)x, (long)ldx, (h16*)y, gamma,
                         beta, rows, C, eps, skip_period);
    else
      hipLaunchKernelGGL(layernorm_narrow_kernel<64>, grid, dim3(256), 0, st, (const h16*)x, (long)ldx, (h16*)y, gamma,
                         beta, rows, C, eps, skip_period);
  } else {
    hipLaunchKernelGGL(layernorm_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, (const h16*)x, (long)ldx, (h16*)y,
                       gamma, beta, rows, C, eps, skip_period);
  }
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int64_t vda_groupnorm_workspace(int32_t F, int32_t S, int32_t C, int32_t groups) {
  if (F <= 0 || S <= 0 || C <= 0 || groups <= 0) return 0;
  const long nchunk = (S + gn_rows(C) - 1) / gn_rows(C);
  return (int64_t)(2L * F * nchunk * C + 2L * F * groups);
}

extern "C" int vda_groupnorm(const void* x, void* y, const float* gamma, const float* beta, int32_t F,
                             int32_t S, int32_t C, int32_t groups, float eps, float* ws, void* stream) {
  VDA_CHECK_ARG(x && y && gamma && beta, "null pointer");
  VDA_CHECK_ARG(F > 0 && S > 0 && groups > 0 && C % groups == 0, "C must be divisible by groups");
  const int cg = C / groups;
  VDA_CHECK_ARG(cg % 2 == 0, "channels per group must be even");
  hipStream_t st = (hipStream_t)stream;
  if (ws && C % 8 == 0 && C <= 2048) {
    const int nchunk = (S + gn_rows(C) - 1) / gn_rows(C);
    float* stats = ws + 2L * F * nchunk * C;
    hipLaunchKernelGGL(gn_partial_kernel, dim3(F * nchunk), dim3(256), 0, st, (const h16*)x, ws, S, C, groups, nchunk);
    hipLaunchKernelGGL(gn_finalize_kernel, dim3(F * groups), dim3(64), 0, st, (const h16*)x, (const float*)ws, stats, S,
                       C, groups, nchunk, eps);
    hipLaunchKernelGGL(gn_apply_kernel, dim3(F * nchunk), dim3(256), 0, st, (const h16*)x, (h16*)y, (const float*)stats,
                       gamma, beta, S, C, groups, nchunk);
    VDA_LAUNCH_CHECK();
    return 0;
  }
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
