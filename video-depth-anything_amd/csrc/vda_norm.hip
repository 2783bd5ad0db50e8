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

__device__ __forceinline__ void gn_partial_block(const h16* __restrict__ x, float* __restrict__ part, int S, int C,
                                                 int groups, int nchunk, int bid, float* red) {
  const int f = bid / nchunk, ch = bid % nchunk;
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

__global__ __launch_bounds__(256) void gn_partial_kernel(const h16* __restrict__ x, float* __restrict__ part, int S, int C,
                                                         int groups, int nchunk) {
  __shared__ float red[256 * 16];  // [thread][sum d x8 | sum d^2 x8] (16 KB)
  gn_partial_block(x, part, S, C, groups, nchunk, blockIdx.x, red);
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
    of[j] = __builtin_fmaf(-mean, sc[j], bet[c]);  // spelled out: gn_linear_kernel forms the same bits
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

// GroupNorm -> Linear (motion_module.py:116-119: norm, rearrange, proj_in) with the normalisation applied
// to the GEMM operand in registers instead of through a normalised copy of x in HBM.  The operand is
// exactly gn_apply's output, z = fp16(fma(x, sc, of)), sc = rstd_fg gamma_c, of = fma(-mean_fg, sc, beta_c),
// so the fused route and the GroupNorm + GEMM composition differ only in the fp32 accumulation order.
// A block (8 waves, one per CU: the weights are resident) stages W [N, K] into LDS once (128 KiB at
// C = 256, 16-B chunks XOR-swizzled by row) with gamma, beta and the bias; each wave streams 16-row
// tiles: per k-step s, lane group q takes the 16-byte chunk 4s + q of its row (one load instruction =
// 64 contiguous bytes of 16 rows), forms z with v_fma_mix_f32 on the packed fp16 pairs, and runs
// v_mfma_f32_16x16x32_f16 with A = W fragments from LDS, B = z; + bias, fp16 8-B stores, optional per-row
// (sum, sum of squares) for a following LN-folded GEMM.  The next tile's x and per-row group statistics
// are loaded before the current tile's MFMAs (two register sets, two waves per SIMD).  Each lane looks up
// its own row's frame, so tiles may span frames (any S).  K = N = C in {64, 128, 256}, 32 groups.
// hipcc's own SLP packing of this transform (v_pk_fma_f32 broadcasting the scale through op_sel) gave
// wrong values on lanes 48-63 for some k-steps on gfx950 (tools/dbg_gnl2.py): the
// v_fma_mix form is spelled out.
// Roofline: HBM (x in, y out: 4 C bytes per row); the W fragment reads (C^2 / 8 bytes of LDS per 16-row
// tile) and the MFMAs stay under it.
constexpr int GNL_GROUPS = 32;
constexpr int GNL_WAVES = 8;

template <int K>
__global__ __launch_bounds__(64 * GNL_WAVES, 1) void gn_linear_kernel(
    const h16* __restrict__ x, const float* __restrict__ stats, const h16* __restrict__ w,
    const float* __restrict__ gam, const float* __restrict__ bet, const float* __restrict__ bias,
    h16* __restrict__ y, float* __restrict__ stats_out, int M, int S, int ntiles) {
  constexpr int N = K;
  constexpr int NTH = 64 * GNL_WAVES;
  constexpr int CH = K / 8;                      // 16-byte chunks per row
  constexpr int KS = K / 32;                     // MFMA k-steps; step s, lane group q: chunk 4s + q
  constexpr int NT = N / 16;                     // 16-column tiles of the output
  constexpr int SWZ = (CH >= 16 ? 16 : CH) - 1;  // chunk XOR of the W rows: 16 lanes, 16 distinct slots
  constexpr int CG = K / GNL_GROUPS;             // channels per group
  constexpr int GPC = 8 / CG;                    // groups per chunk
  __shared__ __attribute__((aligned(16))) h16 sw[N * K];
  __shared__ __attribute__((aligned(16))) float sb[N];
  __shared__ __attribute__((aligned(16))) float sg[K];
  __shared__ __attribute__((aligned(16))) float sbe[K];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  {  // W into LDS with the chunk XOR, every load in flight at once; gamma / beta / bias beside it
    constexpr int R = N * CH / NTH;
    static_assert(N * CH % NTH == 0, "whole staging rounds");
    uint4 wv[R];
#pragma unroll
    for (int it = 0; it < R; ++it) wv[it] = ldg16(w + (long)(tid + it * NTH) * 8);
#pragma unroll
    for (int it = 0; it < R; ++it) {
      const int i = tid + it * NTH, n = i / CH, c = i - n * CH;
      *reinterpret_cast<uint4*>(&sw[n * K + ((c ^ (n & SWZ)) * 8)]) = wv[it];
    }
    if (tid < N) sb[tid] = bias ? bias[tid] : 0.f;
    if (tid < K) {
      sg[tid] = gam[tid];
      sbe[tid] = bet[tid];
    }
  }
  __syncthreads();

  const int q = lane >> 4, r16 = lane & 15;
  const int tstride = gridDim.x * GNL_WAVES;
  int t = blockIdx.x * GNL_WAVES + wave;
  if (t >= ntiles) return;  // no barrier below this point
  const float2* st2 = reinterpret_cast<const float2*>(stats);
  auto load = [&](int tt, uint4 (&xb)[KS], float2 (&sv)[KS][GPC]) {
    const int m = min(tt * 16 + r16, M - 1);
    const h16* xp = x + (long)m * K + q * 8;
    const float2* sp = st2 + (long)(m / S) * GNL_GROUPS + q * GPC;
#pragma unroll
    for (int s = 0; s < KS; ++s) xb[s] = ldg16(xp + s * 32);
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int k = 0; k < GPC; ++k) sv[s][k] = sp[4 * s * GPC + k];
  };
  const h16* wq = sw + r16 * K;
  auto compute = [&](int tt, const uint4 (&xb)[KS], const float2 (&sv)[KS][GPC]) {
    f4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int c8 = (4 * s + q) * 8;  // first channel of this lane's chunk
      const float4 g0 = *reinterpret_cast<const float4*>(&sg[c8]), g1 = *reinterpret_cast<const float4*>(&sg[c8 + 4]);
      const float4 e0 = *reinterpret_cast<const float4*>(&sbe[c8]), e1 = *reinterpret_cast<const float4*>(&sbe[c8 + 4]);
      const float ga[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float be[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
      const unsigned xv[4] = {xb[s].x, xb[s].y, xb[s].z, xb[s].w};
      unsigned zv[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {  // gn_apply's z = fp16(fma(x, sc, of)), the fma on the packed fp16 x
        const float2 m0 = sv[s][(2 * p) / CG], m1 = sv[s][(2 * p + 1) / CG];  // (mean, rstd)
        const float sc0 = mul_f32(m0.y, ga[2 * p]), sc1 = mul_f32(m1.y, ga[2 * p + 1]);
        const float of0 = fma_f32(-m0.x, sc0, be[2 * p]), of1 = fma_f32(-m1.x, sc1, be[2 * p + 1]);
        const float lo = fma_mix_lo(sc0, xv[p], of0);
        const float hi = fma_mix_hi(sc1, xv[p], of1);
        typedef float f2v __attribute__((ext_vector_type(2)));
        zv[p] = __builtin_bit_cast(unsigned, __builtin_convertvector(f2v{lo, hi}, h2));
      }
      const h8 z = __builtin_bit_cast(h8, make_uint4(zv[0], zv[1], zv[2], zv[3]));
      const int cs = ((4 * s + q) ^ (r16 & SWZ)) * 8;
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[j] = mfma16(*reinterpret_cast<const h8*>(wq + j * 16 * K + cs), z, acc[j]);
    }
    // epilogue: lane holds y[m = 16 tt + r16][n = 16j + 4q + i]
    const int m = tt * 16 + r16;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const float4 b = *reinterpret_cast<const float4*>(&sb[j * 16 + 4 * q]);
      h4 o;
      o[0] = (h16)(acc[j][0] + b.x);
      o[1] = (h16)(acc[j][1] + b.y);
      o[2] = (h16)(acc[j][2] + b.z);
      o[3] = (h16)(acc[j][3] + b.w);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float f = (float)o[i];
        s1 += f;
        s2 = fmaf(f, f, s2);
      }
      if (m < M) *reinterpret_cast<h4*>(y + (long)m * N + j * 16 + 4 * q) = o;
    }
    if (stats_out) {  // sum over the 4 lane groups (lane bits 4, 5), then one (sum, sumsq) per row
      float a, b;
      swap16_pair(s1, a, b);
      s1 = half_sum(a + b);
      swap16_pair(s2, a, b);
      s2 = half_sum(a + b);
      if (q == 0 && m < M) *reinterpret_cast<float2*>(stats_out + 2L * m) = make_float2(s1, s2);
    }
  };
  // two register sets, the next tile's loads issued before the current tile's MFMAs; a wave past the
  // end re-reads its own tile (no branch around the loads) and exits after its last store
  uint4 xa[KS], xb[KS];
  float2 sa[KS][GPC], sb2[KS][GPC];
  load(t, xa, sa);
  while (true) {
    const int t1 = t + tstride;
    load(t1 < ntiles ? t1 : t, xb, sb2);
    compute(t, xa, sa);
    if (t1 >= ntiles) break;
    const int t2 = t1 + tstride;
    load(t2 < ntiles ? t2 : t1, xa, sa);
    compute(t1, xb, sb2);
    if (t2 >= ntiles) break;
    t = t2;
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

// ---- GroupNorm -> Linear ------------------------------------------------------------------------
namespace {
bool gnl_fused(int32_t C, int32_t groups, int32_t N) {
  return groups == GNL_GROUPS && N == C && (C == 64 || C == 128 || C == 256);
}
int64_t gnl_stats_bytes(int32_t F, int32_t S, int32_t C, int32_t groups) {
  return (vda_groupnorm_workspace(F, S, C, groups) * 4 + 255) / 256 * 256;
}

}  // namespace

extern "C" int vda_groupnorm_linear_fused(int32_t C, int32_t groups, int32_t N) { return gnl_fused(C, groups, N) ? 1 : 0; }

extern "C" int64_t vda_groupnorm_linear_workspace(int32_t F, int32_t S, int32_t C, int32_t groups, int32_t N) {
  if (F <= 0 || S <= 0 || C <= 0 || groups <= 0 || N <= 0) return 0;
  const int64_t b = gnl_stats_bytes(F, S, C, groups);
  return gnl_fused(C, groups, N) ? b : b + (int64_t)F * S * C * 2;  // + the normalised copy of x (unfused route)
}

extern "C" int vda_groupnorm_linear(const void* x, const float* gamma, const float* beta, int32_t F, int32_t S,
                                    int32_t C, int32_t groups, float eps, const void* w, const float* bias, void* y,
                                    int32_t N, float* stats_out, void* ws, int64_t ws_bytes, void* stream) {
  VDA_CHECK_ARG(x && gamma && beta && w && y && ws, "null pointer");
  VDA_CHECK_ARG(F > 0 && S > 0 && groups > 0 && C % groups == 0 && C % 8 == 0 && C <= 2048 && N > 0,
                "C must be a multiple of 8 and of groups, <= 2048");
  VDA_CHECK_ARG((long)F * S <= 0x7fffffffL, "F * S rows must fit int32");
  VDA_CHECK_ARG(ws_bytes >= vda_groupnorm_linear_workspace(F, S, C, groups, N), "workspace too small");
  VDA_CHECK_ARG((uintptr_t)ws % 16 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)w % 16 == 0 && (uintptr_t)y % 16 == 0,
                "x, w, y and ws must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  const int M = F * S;
  float* wsf = (float*)ws;
  if (!gnl_fused(C, groups, N)) {  // the two-kernel composition: vda_groupnorm into ws, then vda_gemm
    void* xn = (char*)ws + gnl_stats_bytes(F, S, C, groups);
    int rc = vda_groupnorm(x, xn, gamma, beta, F, S, C, groups, eps, wsf, stream);
    if (rc) return rc;
    vda_epilogue e = {};
    e.bias = bias;
    e.rdiv = e.rmod = 1;
    e.stats_out = stats_out;
    return vda_gemm(xn, C, w, y, N, M, N, C, &e, stream);
  }
  const int nchunk = (S + gn_rows(C) - 1) / gn_rows(C);
  float* stats = wsf + 2L * F * nchunk * C;
  const int ntiles = (M + 15) / 16;
  const int nblk = std::min(vda_cu_count(), (ntiles + GNL_WAVES - 1) / GNL_WAVES);
  hipLaunchKernelGGL(gn_partial_kernel, dim3(F * nchunk), dim3(256), 0, st, (const h16*)x, wsf, S, C, groups, nchunk);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(F * groups), dim3(64), 0, st, (const h16*)x, (const float*)wsf, stats, S,
                     C, groups, nchunk, eps);
#define VDA_GNL(KK)                                                                                                 \
  hipLaunchKernelGGL(gn_linear_kernel<KK>, dim3(nblk), dim3(64 * GNL_WAVES), 0, st, (const h16*)x, (const float*)stats, \
                     (const h16*)w, gamma, beta, bias, (h16*)y, stats_out, M, S, ntiles)
  if (C == 256)
    VDA_GNL(256);
  else if (C == 128)
    VDA_GNL(128);
  else
    VDA_GNL(64);
#undef VDA_GNL
  VDA_LAUNCH_CHECK();
  return 0;
}
