// MFMA GEMM + implicit-GEMM convolution with fused epilogues (gfx950).
//
// Y[m, n] = epi( sum_k X[m, k] * W[n, k] ).  One kernel template serves every nn.Linear, 1x1
// conv, ConvTranspose2d(k=s) and 3x3 conv of the Video-Depth-Anything forward (see include/vda.h
// for the reference call sites).
//
// Tiling: BM x BN block tile, BK = 64, 256 threads = 4 waves as 2 (m) x 2 (n); each wave owns a
// (BM/2) x (BN/2) sub-tile computed with v_mfma_f32_16x16x32_f16.  The MFMA is issued in the
// "swapped" orientation: the A operand is a 16-row slice of W (output channels) and the B operand
// a 16-row slice of X (tokens/pixels), so each lane ends up holding FOUR CONSECUTIVE OUTPUT
// CHANNELS of one token: the epilogue does 8-byte loads/stores of bias/residual/output and the
// GEGLU pair (h, g) of a channel lands in the same lane.
//
// Staging: register-staged double-buffered LDS (global loads for tile t+1 are issued before the
// MFMAs of tile t, written to the other LDS buffer after them; one barrier per K tile).  LDS rows
// are 128 B (64 halfs) with the 16-B chunk index XOR-swizzled by (row>>1)&7, which makes both the
// ds_write_b128 stores and the 16-lane ds_read_b128 fragment reads bank-conflict free.
#include "vda_common.h"
#include "phi_table.h"
#include <type_traits>
#ifdef VDA_TS  // phase timestamps of every phased tile (tools/ts_probe2.py; experiments only)
__device__ unsigned long long g_ts[4096][8];
#define TS(k) do { if (threadIdx.x == 0 && vb < 4096) g_ts[vb][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
extern "C" int vda_debug_timestamps(void* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ts), sizeof(g_ts), 0, hipMemcpyDeviceToHost);
}
// per-block clock stamps of the persistent GEMM (tools/clock_probe.py): s_memtime (shader clock) and
// s_memrealtime (100 MHz) at block start and end, so clock = d(memtime) / d(realtime) x 100 MHz
__device__ unsigned long long g_tsc[1024][4];
#define TSC(k) do { if (threadIdx.x == 0 && blockIdx.x < 1024) { \
    g_tsc[blockIdx.x][2 * (k)] = __builtin_amdgcn_s_memtime(); \
    g_tsc[blockIdx.x][2 * (k) + 1] = __builtin_amdgcn_s_memrealtime(); } } while (0)
extern "C" int vda_debug_clock_stamps(void* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tsc), sizeof(g_tsc), 0, hipMemcpyDeviceToHost);
}
#else
#define TS(k) do {} while (0)
#define TSC(k) do {} while (0)
#endif
#include "../../include/vda.h"

// cache policy of the phased epilogue's output stores: nt (aux = 2).  In-situ A/B on one box
// (tools/ab_libs.sh, 2 rounds): every phased GEMM/conv class 0.7-3.6 % faster, the forward's kernel
// sum 55.77 -> 55.33 ms; the output tile is not re-read by the launch, so it need not stay in L2.
constexpr int VDA_EPI_STORE_AUX = 2;

// halo-tiled 3x3 kernels (vda_depth.hip)
int vda_depth_halo(const void* U, const void* w1, const float* b1, const float* w2, const float* b2, float* depth,
                   int BT, int H, int W, int C, hipStream_t st);
int vda_conv_strip(const void* x, const void* w, void* y, const float* bias, int relu_out, int pre_relu,
                   const void* res, const void* res2, int BT, int H, int W, int Cin, int Cout, void* ws,
                   long ws_bytes, hipStream_t st);
bool vda_conv_strip_serves(int W, int Cin, int Cout);
long vda_conv_strip_ws_bytes(int BT, int H, int W, int Cin, int Cout);
bool vda_depth_halo_fused_serves(int Hs, int Ws, int H, int W, int C);
int vda_conv_halo(const void* x, const void* w, void* y, const float* bias, int relu, int BT, int H, int W, int Cin,
                  int Cout, hipStream_t st);
int vda_depth_halo_fused(const void* x, const void* w1, const float* b1, const float* w2, const float* b2,
                         float* depth, int BT, int Hs, int Ws, int H, int W, int C, hipStream_t st);
int vda_conv_halo_fused(const void* x, const void* w, void* y, const float* bias, int relu, int BT, int Hs, int Ws,
                        int H, int W, int Cin, int Cout, hipStream_t st);
// depth-tail conv on the resized map, 2 blocks / CU (vda_dconv.hip)
bool vda_depth_conv_serves(int H, int W, int C);
int vda_depth_conv(const void* U, const void* w1, const float* b1, const float* w2, const float* b2, float* depth,
                   int BT, int H, int W, int C, hipStream_t st);
bool vda_depth_conv_fused_serves(int Hs, int Ws, int H, int W, int C);
int vda_depth_conv_fused(const void* x, const void* w1, const float* b1, const float* w2, const float* b2,
                         float* depth, int BT, int Hs, int Ws, int H, int W, int C, hipStream_t st);
// per-row partial statistics of an fp16 matrix (vda_norm.hip): the stats_out fallback
int vda_row_partials_launch(const void* y, int64_t ldy, float* out, int32_t rows, int32_t N, hipStream_t st);
// halo-tiled phased 3x3 conv, Cout = 256 (vda_hconv.hip)
bool vda_conv_hconv_serves(int BT, int H, int W, int Cin, int Cout);
int vda_conv_im2col(const void* x, void* a, int BT, int H, int W, int Cin, int Ho, int Wo, int ks, int stride, int pad,
                    hipStream_t st);
int vda_conv_hconv(const void* x, const void* w, void* y, const float* bias, int relu_out, int pre_relu,
                   const void* res, const void* res2, int res2_h, int res2_w, int BT, int H, int W, int Cin, int Cout,
                   hipStream_t st);

namespace {

constexpr int BK = 64;

struct GemmParams {
  const h16* x; long ldx;
  const h16* w;
  h16* y; long ldy;
  int M, N, K;
  // implicit conv geometry (conv mode only)
  int H, W, Cin, Ho, Wo, ks, stride, pad, pre_relu, up_h, up_w;
  vda_epilogue epi;
};

__device__ __forceinline__ int swz(int row, int chunk) {  // half offset in a [rows][64] tile
  return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3);
}

// ---- X-tile loaders -------------------------------------------------------------------------
// Dense: X is a row-major [M, K] matrix with row stride ldx.
struct DenseLoader {
  const h16* rowp[4];
  bool rowok[4];
  __device__ void init(const GemmParams& p, int m0, int tid, int nrow_iters) {
    for (int i = 0; i < nrow_iters; ++i) {
      int r = (tid >> 3) + 32 * i;
      int m = m0 + r;
      rowok[i] = m < p.M;
      rowp[i] = p.x + (long)(rowok[i] ? m : 0) * p.ldx;
    }
  }
  __device__ uint4 load(const GemmParams& p, int i, int k) const {
    if (rowok[i] && k < p.K) return ldg16(rowp[i] + k);
    return make_uint4(0, 0, 0, 0);
  }
};

// Implicit GEMM conv: row m = output pixel (bt, oy, ox), k = (ky*ks + kx)*Cin + ci.
struct ConvLoader {
  int bt[4], oy[4], ox[4];
  bool rowok[4];
  __device__ void init(const GemmParams& p, int m0, int tid, int nrow_iters) {
    for (int i = 0; i < nrow_iters; ++i) {
      int r = (tid >> 3) + 32 * i;
      int m = m0 + r;
      rowok[i] = m < p.M;
      int mm = rowok[i] ? m : 0;
      ox[i] = mm % p.Wo;
      int t = mm / p.Wo;
      oy[i] = t % p.Ho;
      bt[i] = t / p.Ho;
    }
  }
  __device__ uint4 load(const GemmParams& p, int i, int k) const {
    if (!rowok[i] || k >= p.K) return make_uint4(0, 0, 0, 0);
    int tap = k / p.Cin;
    int ci = k - tap * p.Cin;
    int ky = tap / p.ks, kx = tap - ky * p.ks;
    int iy = oy[i] * p.stride - p.pad + ky;
    int ix = ox[i] * p.stride - p.pad + kx;
    uint4 v;
    if (p.up_h > 0) {
      // conv input = bilinear(align_corners=True) upsample of the stored [H, W] map to [up_h, up_w]
      if (iy < 0 || iy >= p.up_h || ix < 0 || ix >= p.up_w) return make_uint4(0, 0, 0, 0);
      float sy = p.up_h > 1 ? (float)(p.H - 1) / (float)(p.up_h - 1) : 0.f;
      float sx = p.up_w > 1 ? (float)(p.W - 1) / (float)(p.up_w - 1) : 0.f;
      float fy = sy * iy, fx = sx * ix;
      int y0 = (int)fy, x0 = (int)fx;
      int y1 = min(y0 + 1, p.H - 1), x1 = min(x0 + 1, p.W - 1);
      float wy = ac_weight(sy, (float)iy, y0), wx = ac_weight(sx, (float)ix, x0);
      const h16* base = p.x + (long)bt[i] * p.H * p.W * p.Cin + ci;
      h8 a = __builtin_bit_cast(h8, ldg16(base + ((long)y0 * p.W + x0) * p.Cin));
      h8 b = __builtin_bit_cast(h8, ldg16(base + ((long)y0 * p.W + x1) * p.Cin));
      h8 c = __builtin_bit_cast(h8, ldg16(base + ((long)y1 * p.W + x0) * p.Cin));
      h8 d = __builtin_bit_cast(h8, ldg16(base + ((long)y1 * p.W + x1) * p.Cin));
      h8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float top = (float)a[j] + ((float)b[j] - (float)a[j]) * wx;
        float bot = (float)c[j] + ((float)d[j] - (float)c[j]) * wx;
        o[j] = (h16)(top + (bot - top) * wy);
      }
      v = __builtin_bit_cast(uint4, o);
    } else {
      if (iy < 0 || iy >= p.H || ix < 0 || ix >= p.W) return make_uint4(0, 0, 0, 0);
      v = ldg16(p.x + (((long)bt[i] * p.H + iy) * p.W + ix) * p.Cin + ci);
    }
    if (p.pre_relu) v = relu_h8(v);
    return v;
  }
};

// ---- epilogue ------------------------------------------------------------------------------
// LayerNorm folded into the GEMM (vda_epilogue.ln_stats / ln_colsum): the row's (mean, rstd), from
// [M, 2] as is or from [M, ln_parts, 2] partial (sum, sumsq) over ln_parts column blocks
__device__ __forceinline__ float2 epi_ln_row(const GemmParams& p, int m) {
  const vda_epilogue& e = p.epi;
  if (e.ln_parts > 0) {
    float sm = 0.f, sq = 0.f;
    for (int t = 0; t < e.ln_parts; ++t) {
      const float2 pq = *reinterpret_cast<const float2*>(e.ln_stats + 2L * ((long)m * e.ln_parts + t));
      sm += pq.x;
      sq += pq.y;
    }
    const float mean = sm / (float)p.K;
    return make_float2(mean, rsqrtf(fmaxf(fmaf(-mean, mean, sq / (float)p.K), 0.f) + e.ln_eps));
  }
  return *reinterpret_cast<const float2*>(e.ln_stats + 2L * m);
}
template <int ACT>
__device__ __forceinline__ void epi_store4(const GemmParams& p, int m, int n, f4 v) {
  const vda_epilogue& e = p.epi;
  if (e.ln_stats) {  // LayerNorm folded into the GEMM: rstd * (acc - mean * colsum)
    const float2 mr = epi_ln_row(p, m);
    const f4 c1 = *reinterpret_cast<const f4*>(e.ln_colsum + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = mr.y * fmaf(-mr.x, c1[j], v[j]);
  }
  if (e.bias) {
    f4 b = *reinterpret_cast<const f4*>(e.bias + n);
    v += b;
  }
  if (e.rowbias) {
    int r = (m / e.rdiv) % e.rmod;
    f4 b = *reinterpret_cast<const f4*>(e.rowbias + (long)r * p.N + n);
    v += b;
  }
  if constexpr (ACT == VDA_ACT_GELU) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = gelu_erf(v[j]);
  } else if constexpr (ACT == VDA_ACT_RELU) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
  }
  if (e.gamma) {
    f4 g = *reinterpret_cast<const f4*>(e.gamma + n);
    v *= g;
  }
  if (e.res) {
    h4 r = *reinterpret_cast<const h4*>((const h16*)e.res + (long)m * e.ldres + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += (float)r[j];
  }
  if (e.res2) {
    h4 r = *reinterpret_cast<const h4*>((const h16*)e.res2 + (long)m * e.ldres2 + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += (float)r[j];
  }
  h4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = (h16)v[j];
  long off;
  if (e.store == VDA_STORE_PIXEL_SHUFFLE) {
    int k = e.ps_k, cout = e.ps_cout;
    int ij = n / cout, co = n - ij * cout;
    int ki = ij / k, kj = ij - ki * k;
    int xw = m % e.ps_win;
    int t = m / e.ps_win;
    int yh = t % e.ps_hin;
    int bt = t / e.ps_hin;
    long oh = (long)yh * k + ki, ow = (long)xw * k + kj;
    off = (((long)bt * e.ps_hin * k + oh) * ((long)e.ps_win * k) + ow) * cout + co;
  } else {
    off = (long)m * p.ldy + n;
  }
  *reinterpret_cast<h4*>(p.y + off) = o;
}

// GEGLU: h and g accumulators for the same 4 output channels.  Output column = n_out.
__device__ __forceinline__ void epi_geglu4(const GemmParams& p, int m, int nh, int ng, int n_out,
                                           f4 vh, f4 vg) {
  const vda_epilogue& e = p.epi;
  if (e.ln_stats) {  // LayerNorm folded in (the motion modules' ff_norm), on both halves before the gate
    const float2 mr = epi_ln_row(p, m);
    const f4 ch = *reinterpret_cast<const f4*>(e.ln_colsum + nh), cg = *reinterpret_cast<const f4*>(e.ln_colsum + ng);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      vh[j] = mr.y * fmaf(-mr.x, ch[j], vh[j]);
      vg[j] = mr.y * fmaf(-mr.x, cg[j], vg[j]);
    }
  }
  if (e.bias) {
    vh += *reinterpret_cast<const f4*>(e.bias + nh);
    vg += *reinterpret_cast<const f4*>(e.bias + ng);
  }
  f4 v;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = vh[j] * gelu_erf(vg[j]);
  const int nout_tot = p.N >> 1;
  if (e.gamma) v *= *reinterpret_cast<const f4*>(e.gamma + n_out);
  if (e.res) {
    h4 r = *reinterpret_cast<const h4*>((const h16*)e.res + (long)m * e.ldres + n_out);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += (float)r[j];
  }
  (void)nout_tot;
  h4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = (h16)v[j];
  *reinterpret_cast<h4*>(p.y + (long)m * p.ldy + n_out) = o;
}

// ---- register-staged kernel (conv with a fused bilinear-upsample loader) ----------------------
template <int BM, int BN, class Loader, int ACT>
__global__ __launch_bounds__(256) void gemm_reg_kernel(GemmParams p, int tiles_n) {
  constexpr int TM = BM / 32;  // 16-row m subtiles per wave
  constexpr int TN = BN / 32;  // 16-row n subtiles per wave
  constexpr int XIT = BM / 32; // 16-B chunks per thread for the X tile (BM*8 / 256)
  constexpr int WIT = BN / 32;
  __shared__ __attribute__((aligned(16))) h16 sX[2][BM * BK];
  __shared__ __attribute__((aligned(16))) h16 sW[2][BN * BK];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int tile_n = blockIdx.x % tiles_n, tile_m = blockIdx.x / tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  Loader ld;
  ld.init(p, m0, tid, XIT);
  const h16* wrow[WIT];
  bool wok[WIT];
#pragma unroll
  for (int i = 0; i < WIT; ++i) {
    int n = n0 + (tid >> 3) + 32 * i;
    wok[i] = n < p.N;
    wrow[i] = p.w + (long)(wok[i] ? n : 0) * p.K;
  }
  const int cchunk = tid & 7;

  uint4 rx[XIT], rw[WIT];
  auto gload = [&](int k0) {
    int k = k0 + cchunk * 8;
#pragma unroll
    for (int i = 0; i < XIT; ++i) rx[i] = ld.load(p, i, k);
#pragma unroll
    for (int i = 0; i < WIT; ++i) rw[i] = (wok[i] && k < p.K) ? ldg16(wrow[i] + k) : make_uint4(0, 0, 0, 0);
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XIT; ++i) *reinterpret_cast<uint4*>(&sX[buf][swz((tid >> 3) + 32 * i, cchunk)]) = rx[i];
#pragma unroll
    for (int i = 0; i < WIT; ++i) *reinterpret_cast<uint4*>(&sW[buf][swz((tid >> 3) + 32 * i, cchunk)]) = rw[i];
  };

  f4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  gload(0);
  sstore(0);
  __syncthreads();

  const int frow = lane & 15, fchunk = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      h8 af[TN], bf[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i)
        af[i] = *reinterpret_cast<const h8*>(&sW[buf][swz(wn * (BN / 2) + i * 16 + frow, ks * 4 + fchunk)]);
#pragma unroll
      for (int j = 0; j < TM; ++j)
        bf[j] = *reinterpret_cast<const h8*>(&sX[buf][swz(wm * (BM / 2) + j * 16 + frow, ks * 4 + fchunk)]);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds D[n = 4*(lane>>4) + r][m = lane&15] of every (i, j) subtile
  const int mcol = lane & 15, nq = (lane >> 4) * 4;
  if constexpr (ACT == VDA_ACT_GEGLU) {
#pragma unroll
    for (int i = 0; i < TN; i += 2) {
      const int nbase = n0 + wn * (BN / 2) + i * 16;  // h block; gate block = nbase + 16
      if (nbase >= p.N) continue;
      const int n_out = (nbase >> 1) + nq;
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        int m = m0 + wm * (BM / 2) + j * 16 + mcol;
        if (m < p.M) epi_geglu4(p, m, nbase + nq, nbase + 16 + nq, n_out, acc[i][j], acc[i + 1][j]);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int n = n0 + wn * (BN / 2) + i * 16 + nq;
      if (n >= p.N) continue;
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        int m = m0 + wm * (BM / 2) + j * 16 + mcol;
        if (m < p.M) epi_store4<ACT>(p, m, n, acc[i][j]);
      }
    }
  }
}

// ---- LDS-DMA kernel (every dense GEMM and plain conv) ------------------------------------------
// Operand tiles are moved HBM -> LDS with global_load_lds_dwordx4 (no VGPR staging): one wave
// instruction fills 8 rows x 128 B of the [BM + BN][64] tile (X rows first, then W rows).  The DMA
// destination is lane-linear, so the (row>>1)&7 chunk swizzle is applied to the per-lane SOURCE
// address.  Lanes whose source is out of range (rows >= M / N, k >= K, conv zero padding) read a
// zero page instead, so no predication reaches the LDS image.  Two LDS buffers, BK = 64: tile t+1
// is issued before the MFMAs of tile t and drained by the barrier that ends tile t.
// Block -> tile mapping is XCD-aware: the 8 XCDs each take a contiguous run of tiles, grouped
// GROUP_M m-panels at a time so co-resident blocks share X panels and W tiles in their XCD's L2.
__device__ __attribute__((aligned(64))) uint4 g_zero_page[4];

#ifndef VDA_GROUP_M  // (A/B builds only)
#define VDA_GROUP_M 8
#endif
constexpr int GROUP_M = VDA_GROUP_M;  // m-panels per XCD tile group (2 / 4 / 16 within noise: profiles/r04_ab_gemm_group_m.log)
constexpr int ACT_DEPTH = 4;  // internal: depth-head tail epilogue (vda_depth_head)

__device__ __forceinline__ void tile_coords(int bid, int nwg, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - group * per_group;
  tm = first_m + in_group % gsize;
  tn = in_group / gsize;
}

// gelu(x) = x * Phi(x), Phi from the LDS copy of phi_table.h: 2,048 lines A_i + B_i x, one per
// 1/128-wide interval centred on x_i = -8 + i/128 (clamped outside [-8, 8]), |error| <= 1.3e-6
// absolute, far below the fp16 output rounding.  The interval is picked by the magic add
// v = x*128 + (1.5*2^23 + 1024), whose low mantissa bits are round(x*128) + 1024; its byte offset
// (bits << 3, wrapping the exponent bits away) feeds one 8-byte LDS read of {A_i, B_i}, so a value
// costs fma + med3 + shift-add + fma + mul (the erf form needs a v_rcp and a v_exp per element;
// round 1's interpolating table needed a cvt and a fract more).
constexpr float PHI_MAGIC = 12583936.f;                        // 1.5 * 2^23 + 1024
constexpr float PHI_LO = 12582912.f, PHI_HI = 12584959.f;      // node 0 and node 2047
constexpr unsigned PHI_BIAS = 0x4B400000u << 3;                // bits(1.5 * 2^23) * 8 (mod 2^32)
constexpr int PHI_LDS_HALVES = 8192;                           // 16 KiB of LDS
typedef float phi_f2 __attribute__((ext_vector_type(2)));
typedef VDA_LDS const phi_f2* lds_cf2p;
__device__ __forceinline__ unsigned phi_base(const float* tab) {
  return (unsigned)(uintptr_t)(VDA_LDS const float*)tab - PHI_BIAS;
}
__device__ __forceinline__ phi_f2 phi_line(float x, unsigned phib) {
  const float v = __builtin_amdgcn_fmed3f(fmaf(x, 128.f, PHI_MAGIC), PHI_LO, PHI_HI);
  return *(lds_cf2p)(uintptr_t)((__builtin_bit_cast(unsigned, v) << 3) + phib);
}

// LDS float2 access through asm (hipcc inserts no LDS-DMA alias wait for it); the read waits for itself
__device__ __forceinline__ float2 lds_ld_f2(const float* ptr) {
  float2 v;
  asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v)
               : "v"((unsigned)(uintptr_t)(VDA_LDS const float*)ptr) : "memory");
  return v;
}
__device__ __forceinline__ void lds_ld_f4x2(const float* ptr, float4& a, float4& b) {
  // early-clobber outputs: the second read must not take its address from the first read's destination
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)" : "=&v"(a), "=&v"(b)
               : "v"((unsigned)(uintptr_t)(VDA_LDS const float*)ptr) : "memory");
}
__device__ __forceinline__ float lds_ld_f1(const float* ptr) {
  float v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v)
               : "v"((unsigned)(uintptr_t)(VDA_LDS const float*)ptr) : "memory");
  return v;
}
__device__ __forceinline__ void lds_st_f2(float* ptr, float2 v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"((unsigned)(uintptr_t)(VDA_LDS float*)ptr), "v"(v) : "memory");
}

// Dynamic tile schedule (vda_epilogue.sched): one agent-scope ticket draw per tile, through asm so that
// the compiler's vmcnt bookkeeping never waits for it (the counted DMA waits that follow retire it: it is
// older than the pieces they leave in flight), and the slot it is published to in LDS.
__device__ __forceinline__ unsigned ticket_draw(unsigned* ctr) {
  unsigned v;
  asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(v) : "v"(ctr), "v"(1u) : "memory");
  return v;
}
// publishes tile base + 8 v; v (the draw's asm output) is read only inside this asm, after the counted
// wait that retired the draw, so no compiler-scheduled use of it can run before the value has landed
__device__ __forceinline__ void ticket_publish(int* ptr, unsigned v, int base) {
  unsigned t;
  asm volatile("v_lshl_add_u32 %0, %1, 3, %2\n\tds_write_b32 %3, %0" : "=&v"(t)
               : "v"(v), "s"(base), "v"((unsigned)(uintptr_t)(VDA_LDS int*)ptr) : "memory");
}
__device__ __forceinline__ int lds_ld_i1(const int* ptr) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v)
               : "v"((unsigned)(uintptr_t)(VDA_LDS const int*)ptr) : "memory");
  return v;
}

__device__ __forceinline__ void glds16(const void* src, h16* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (VDA_LDS void*)lds_base, 16, 0, 0);
}

template <int KB>
__device__ __forceinline__ int swzk(int row, int chunk) {  // half offset in a [rows][KB] tile
  constexpr int CH = KB / 8;
  return row * KB + ((chunk ^ ((row >> 1) & (CH - 1))) << 3);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// NS-stage LDS-DMA pipeline: tile kt+NS-1 is issued while tile kt is multiplied; before reading a
// stage every wave waits with a COUNTED vmcnt (its own newer pieces stay in flight) and passes a
// raw s_barrier (no __syncthreads: its fence would drain every DMA in flight).
template <int BM, int BN, int NWM, int NWN, int KB, int NS, bool CONV, int ACT>
__global__ __launch_bounds__(NWM * NWN * 64) void gemm_kernel(GemmParams p, int tiles_m, int tiles_n) {
  constexpr int NW = NWM * NWN;
  constexpr int WTM = BM / NWM, WTN = BN / NWN;  // wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int ROWS = BM + BN;
  constexpr int CH = KB / 8;                     // 16-B chunks per row
  constexpr int RPP = 64 / CH;                   // rows per 1-KiB DMA piece
  constexpr int GROUPS = ROWS / RPP;             // pieces per stage
  static_assert(GROUPS % NW == 0, "pieces must divide evenly over the waves");
  constexpr int IPW = GROUPS / NW;               // DMA instructions per wave per stage
  constexpr int STAGE = ROWS * KB;               // halfs per stage
  __shared__ __attribute__((aligned(1024))) h16 smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % NWM, wn = wave / NWM;
  int tile_m, tile_n;
  tile_coords(blockIdx.x, gridDim.x, tiles_m, tiles_n, tile_m, tile_n);
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  // per-lane source descriptors for this wave's IPW pieces
  const h16* rowp[IPW];
  int kch[IPW];        // logical k offset (halfs) of this lane's chunk within the K tile
  bool isx[IPW];
  int cbt[IPW], coy[IPW], cox[IPW];
  bool rowok[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int g = wave * IPW + i;
    const int R = g * RPP + lane / CH;
    const int c = (lane % CH) ^ ((R >> 1) & (CH - 1));
    kch[i] = c * 8;
    isx[i] = R < BM;
    if (R < BM) {
      const int m = m0 + R;
      rowok[i] = m < p.M;
      if constexpr (CONV) {
        const int mm = rowok[i] ? m : 0;
        cox[i] = mm % p.Wo;
        const int t = mm / p.Wo;
        coy[i] = t % p.Ho;
        cbt[i] = t / p.Ho;
        rowp[i] = p.x;
      } else {
        rowp[i] = p.x + (long)(rowok[i] ? m : 0) * p.ldx;
      }
    } else {
      const int n = n0 + R - BM;
      rowok[i] = n < p.N;
      rowp[i] = p.w + (long)(rowok[i] ? n : 0) * p.K;
    }
  }
  const void* zero = (const void*)g_zero_page;

  auto issue = [&](int k0, int buf) {
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int k = k0 + kch[i];
      const void* src = zero;
      if (rowok[i] && k < p.K) {
        if (CONV && isx[i]) {
          const int tap = k / p.Cin, ci = k - tap * p.Cin;
          const int ky = tap / p.ks, kx = tap - ky * p.ks;
          const int iy = coy[i] * p.stride - p.pad + ky, ix = cox[i] * p.stride - p.pad + kx;
          if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W)
            src = p.x + (((long)cbt[i] * p.H + iy) * p.W + ix) * p.Cin + ci;
        } else {
          src = rowp[i] + k;
        }
      }
      glds16(src, smem + buf * STAGE + (wave * IPW + i) * RPP * KB);
    }
  };

  f4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + KB - 1) / KB;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s * KB, s);
  const int frow = lane & 15, fchunk = lane >> 4;
  const bool prerelu = CONV && p.pre_relu;
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt must have landed; the (up to NS-2) newer tiles may stay in flight
    const int newer = min(NS - 2, nk - 1 - kt);
    if constexpr (NS >= 4) {
      if (newer >= 2) wait_vmcnt<2 * IPW>();
      else if (newer == 1) wait_vmcnt<IPW>();
      else wait_vmcnt<0>();
    } else if constexpr (NS == 3) {
      if (newer >= 1) wait_vmcnt<IPW>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    {
      const int nxt = kt + NS - 1;
      if (nxt < nk) issue(nxt * KB, nxt % NS);
    }
    const h16* sX = smem + buf * STAGE;
    const h16* sW = sX + BM * KB;
#pragma unroll
    for (int ks = 0; ks < KB / 32; ++ks) {
      h8 af[TN], bf[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i)
        af[i] = *reinterpret_cast<const h8*>(&sW[swzk<KB>(wn * WTN + i * 16 + frow, ks * 4 + fchunk)]);
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        bf[j] = *reinterpret_cast<const h8*>(&sX[swzk<KB>(wm * WTM + j * 16 + frow, ks * 4 + fchunk)]);
        if (prerelu) bf[j] = relu8(bf[j]);
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
    }
    buf = (buf + 1 == NS) ? 0 : buf + 1;
  }

  const int mcol = lane & 15, nq = (lane >> 4) * 4;
  if constexpr (ACT == ACT_DEPTH) {
    // depth tail (dpt.py:118-124): the wave owns all 64 W rows = 32 output channels as fp16
    // hi (rows 0..31) + lo (rows 32..63) halves of the fp32 weights, so y = acc_hi + acc_lo is the
    // fp32-weight conv.  Then +b1, ReLU, 1x1 (32 -> 1) dot, +b2, ReLU; fp32 depth per pixel.
    static_assert(TN == 4 && NWN == 1, "depth epilogue needs the whole 64-row W tile per wave");
    const float* b1 = p.epi.bias;
    const float* w2 = p.epi.gamma;
    const float b2 = p.epi.rowbias[0];
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      float part = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = i * 16 + nq + r;
          const float y = acc[i][j][r] + acc[i + 2][j][r] + b1[c];
          part += fmaxf(y, 0.f) * w2[c];
        }
      part += __shfl_xor(part, 16, 64);
      part += __shfl_xor(part, 32, 64);
      const int m = m0 + wm * WTM + j * 16 + mcol;
      if (lane < 16 && m < p.M) reinterpret_cast<float*>(p.y)[m] = fmaxf(part + b2, 0.f);
    }
  } else if constexpr (ACT == VDA_ACT_GEGLU) {
    static_assert(TN % 2 == 0, "GEGLU needs an even number of n subtiles per wave");
#pragma unroll
    for (int i = 0; i < TN; i += 2) {
      const int nbase = n0 + wn * WTN + i * 16;
      if (nbase >= p.N) continue;
      const int n_out = (nbase >> 1) + nq;
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0 + wm * WTM + j * 16 + mcol;
        if (m < p.M) epi_geglu4(p, m, nbase + nq, nbase + 16 + nq, n_out, acc[i][j], acc[i + 1][j]);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int n = n0 + wn * WTN + i * 16 + nq;
      if (n >= p.N) continue;
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0 + wm * WTM + j * 16 + mcol;
        if (m < p.M) epi_store4<ACT>(p, m, n, acc[i][j]);
      }
    }
  }
}

// ---- per-row partial statistics in the epilogue (vda_epilogue.stats_out) ----------------------
// A half-wave (32 lanes) owns one output row per phase-2 iteration, 8 columns per lane.  Each lane
// accumulates (sum, sum of squares) of its 8 fp16 outputs with v_dot2_f32_f16 for all 16 rows, then
// one multi-value butterfly over the half-wave leaves lane l with value l of the 32: sum (l & 16 == 0)
// or sum of squares of row 16 * (l & 15).  Step 1 exchanges whole register pairs with
// v_permlane16_swap (no selects); steps 2-5 pair lanes i / 15 - i, 7 - i, 3 - i, i ^ 1 by DPP.
__device__ __forceinline__ void perm16_swap(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float halfwave_sum32(float (&v)[32], int lane) {
  float w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    float a = v[k], b = v[16 + k];
    perm16_swap(a, b);
    w[k] = a + b;
  }
  const int i = lane & 15;
  float x[8], y[4], z[2];
  bool lo = i < 8;
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = (lo ? w[k] : w[k + 8]) + dpp_f<0x140>(lo ? w[k + 8] : w[k]);  // row_mirror
  lo = (i & 7) < 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) y[k] = (lo ? x[k] : x[k + 4]) + dpp_f<0x141>(lo ? x[k + 4] : x[k]);  // row_half_mirror
  lo = (i & 3) < 2;
#pragma unroll
  for (int k = 0; k < 2; ++k) z[k] = (lo ? y[k] : y[k + 2]) + dpp_f<0x1B>(lo ? y[k + 2] : y[k]);  // quad_perm 3,2,1,0
  lo = (i & 1) == 0;
  return (lo ? z[0] : z[1]) + dpp_f<0xB1>(lo ? z[1] : z[0]);  // quad_perm 1,0,3,2
}
__device__ __forceinline__ void stat_acc(h8 t, float& s, float& q) {
  const h2 one = h2{(h16)1.f, (h16)1.f};
  h2 tp[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) tp[k] = h2{t[2 * k], t[2 * k + 1]};
  s = 0.f;
  q = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    s = __builtin_amdgcn_fdot2(tp[k], one, s, false);
    q = __builtin_amdgcn_fdot2(tp[k], tp[k], q, false);
  }
}

// ---- 256x256 phased kernel -------------------------------------------------------------------
// 8 waves (2 m x 4 n), wave tile 128 (m) x 64 (n), BK = 64, two K-tile buffers of four 16-KiB
// half-tile regions [XL | XH | WL | WH].  Every K tile runs as 4 phases; each phase multiplies one
// 64 x 32 quadrant of the wave tile (16 MFMAs) between two barriers, loading the fragments it needs
// (quadrant order (0,0) (0,1) (1,1) (1,0) reuses the previous phase's X or W fragments):
//   P1: ds_read X(q0) + W(q0); DMA XL, XH of tile t+1 | P2: ds_read W(q1); DMA WL, WH of tile t+1
//   P3: ds_read X(q1)                                 | P4: ds_read W(q0); s_waitcnt vmcnt(0)
// Waves 4-7 run one barrier behind waves 0-3, so the two waves sharing a SIMD alternate between
// their LDS-read segment and their MFMA segment.  Restaging a region is >= 2 phases after its
// last read and the DMA wait is one phase before the first read of the new tile (the margins the
// stagger needs).  Raw s_barrier + explicit waits only: nothing drains the DMA queue implicitly.
// Output stores per lane of the row-store epilogue (phase 2): the minimum number of vector-memory
// operations a tile issues after it has pre-issued the next tile's prologue DMA.
template <int XR, int WR, int ACT>
constexpr int phased_nit() {
  constexpr int OW = (ACT == VDA_ACT_GEGLU) ? 64 * WR : 128 * WR;
  return (128 * XR) / (512 / (OW / 8));
}

// Persistent dense tiles chain their prologues: the row-store epilogue of tile t reads its staged
// output back into registers, passes one barrier and then issues tile t+1's prologue DMA (operand
// K tiles 0 and 1, LN statistics) BEFORE its own output stores, so the stores drain under the next
// tile's prologue wait instead of a full vmcnt(0) at the end of every tile (pre = this tile's
// prologue was issued that way; vb_next = the tile this block runs next, or -1).
// EK: compile-time epilogue kind.  0 reads every option of p.epi at run time; 1 = bias (required),
// no gamma / residual / statistics, row store (qkv, fc1 with their LN fold); 2 = bias + one
// residual + row statistics, row store (proj, fc2).  The fixed kinds carry no runtime branches on
// the epilogue, which keeps the uniform state of the persistent loop in SGPRs (no spill reloads,
// whose vmcnt(0) would drain the chained stores at every tile start).
template <int XR, int WR, bool CONV, int ACT, bool ROWB, bool LNF, int EK>  // X / W operand regions of 128 rows (BM = 128 XR, BN = 128 WR)
__device__ __forceinline__ int gemm256_tile(const GemmParams& p, int vb, int tiles_m, int tiles_n, h16* smem,
                                            bool pre, int vb_next, int wave_in, unsigned* tctr = nullptr,
                                            int tbase = 0, int* tslot = nullptr) {
  // vb_next: the static successor (vb + grid, or -1).  tctr: dynamic schedule (this block's XCD ticket
  // counter): wave 0 draws ticket v in K step 0's P3 and publishes tile tbase + 8 v in *tslot after that
  // step's P4 wait; every wave reads it after the main loop.  Returns the tile this block runs next (or -1);
  // only the fixed-kind epilogues (EK != 0) chain its prologue.
  // ROWB: per-row bias support (a separate instantiation: its row-index division would otherwise
  // raise the register pressure of every phased GEMM past the spill point)
  // LNF: LayerNorm folded into the GEMM (vda_epilogue.ln_stats / ln_colsum): X is the raw residual
  // stream, W = gamma (.) W_ln, and the epilogue applies rstd * (acc - mean * colsum) + bias.  The
  // tile's 256 (mean, rstd) pairs are staged into LDS by the prologue DMA (2 KiB after the operand
  // buffers and the Phi table); colsum takes the prefetched gamma registers (gamma is not allowed).
  static_assert(!(LNF && (ROWB || CONV)), "LNF: dense, no row bias");
  static_assert(EK == 0 || (!CONV && !ROWB), "fixed epilogue kinds: dense, no row bias");
  static_assert(EK != 2 || (ACT == VDA_ACT_NONE && !LNF), "EK 2: no activation, no LN fold");
  static_assert(EK != 3 || (ACT == VDA_ACT_NONE && LNF), "EK 3: LN fold + per-frame row bias, no activation");
  const bool has_bias = EK ? true : p.epi.bias != nullptr;
  const bool has_gamma = EK ? false : p.epi.gamma != nullptr;
  // ConvTranspose(k = s) pixel-shuffle stores through the staged row epilogue when a 256-wide N tile is
  // 256 consecutive channels of ONE output pixel (cout % 256 == 0): its rows are then whole 512-B output
  // pixel runs at remapped addresses (phase 2 below), instead of 8-byte scatter stores per element
  // (WR == 2: a 256-wide N tile, 16 rows per store iteration, the only shape ps_store is compiled for; the
  // 16-B row-run stores need a 16-B aligned y)
  const bool ps_rows = !EK && ACT != VDA_ACT_GEGLU && !ROWB && XR == 2 && WR == 2 &&
                       p.epi.store == VDA_STORE_PIXEL_SHUFFLE && p.epi.ps_cout % 256 == 0 && p.epi.ps_win >= 16 &&
                       (long)p.M * p.N * 2 < 0x7fffffffL && (uintptr_t)p.y % 16 == 0;
  const bool rows_store = EK ? true : (p.epi.store == VDA_STORE_ROWS || ps_rows);
  const bool has_res = EK == 2 ? true : (EK == 1 || EK == 3) ? false : p.epi.res != nullptr;
  const bool has_res2 = EK ? false : p.epi.res2 != nullptr;
  const bool has_stats = EK == 2 ? true : (EK == 1 || EK == 3) ? false : p.epi.stats_out != nullptr;
  static_assert(XR * WR == 4 && (XR == 2 || XR == 4), "8 waves as XR (m) x 8/XR (n), wave tile 128 x 64");
  constexpr int BM = 128 * XR, BN = 128 * WR;
  constexpr int HALF = 128 * BK;            // halfs per 128-row region (16 KiB)
  constexpr int BUF = (XR + WR) * HALF;     // one K tile
  // GELU / GEGLU epilogues read Phi from a 16-KiB LDS table (phi_table.h) staged in the prologue
  constexpr bool TAB = XR == 2 && (ACT == VDA_ACT_GELU || ACT == VDA_ACT_GEGLU);
  const float* phi_lds = reinterpret_cast<const float*>(smem + 2 * BUF);
  const unsigned phib = phi_base(phi_lds);
  h16* lnst_lds = smem + 2 * BUF + (TAB ? PHI_LDS_HALVES : 0);  // LNF: [256][2] fp32 (mean, rstd)
  // LNF: tile row whose last statistics entry sits 2 floats further on in LDS (the global array's
  // final entry when M * P is odd: its piece was read 8 B early, see lnst_dma), or -1
  auto lnst_shift_row = [&](int m0_) {
    const int P1 = p.epi.ln_parts > 0 ? p.epi.ln_parts : 1;
    return ((p.M * P1) & 1) && p.M - 1 - m0_ < 256 ? p.M - 1 - m0_ : -1;
  };

  // lane id rebuilt per tile by a volatile mbcnt (and the wave index passed in an SGPR): every
  // lane-derived address below is recomputed per tile instead of being hoisted out of the persistent
  // tile loop, and threadIdx (v0) need not stay live across it (its spill reload's vmcnt(0) at the
  // loop head would drain the chained prologue DMA and stores)
  int lane, wave;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  asm volatile("s_mov_b32 %0, %1" : "=s"(wave) : "s"(wave_in));
  const int tid = wave * 64 + lane;
  const int wm = wave % XR, wn = wave / XR;
  int tile_m, tile_n;
  tile_coords(vb, tiles_m * tiles_n, tiles_m, tiles_n, tile_m, tile_n);
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  // DMA quarters: every operand region is staged as two quarters, each refilled in its own phase
  // (the rows one quadrant of the wave tiles reads).  X quarter i = rows 64i..64i+63 of every X
  // region, W quarter i = rows {32i..32i+31, 64+32i..64+32i+31} of every W region; in each, wave
  // w moves one 8-row piece (1 KiB) per region: this lane's row is xr_of(i) / wr_of(i).
  const h16* xrow[XR][2];
  const h16* wrow[WR][2];
  bool xok[XR][2], wok[WR][2];
  auto xr_of = [&](int i) { return i * 64 + wave * 8 + (lane >> 3); };
  auto wr_of = [&](int i) { return (wave >> 2) * 64 + i * 32 + (wave & 3) * 8 + (lane >> 3); };
  // row bits 0-3 are (wave & 1, lane >> 3) for both layouts, so the source swizzle is one value
  const int kch0 = ((lane & 7) ^ ((((wave & 1) << 3 | (lane >> 3)) >> 1) & 7)) * 8;
  int cyx[XR][2];  // conv: top-left input (row << 16 | col & 0xffff) of the output pixel's window
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int hh = 0; hh < XR; ++hh) {
      const int m = m0 + hh * 128 + xr_of(i);
      xok[hh][i] = m < p.M;
      const int mm = xok[hh][i] ? m : 0;
      if constexpr (CONV) {
        const int ox = mm % p.Wo;
        const int t = mm / p.Wo;
        const int oy = t % p.Ho, bt = t / p.Ho;
        const int iy0 = xok[hh][i] ? oy * p.stride - p.pad : -32768;  // invalid rows fail every bound
        const int ix0 = ox * p.stride - p.pad;
        cyx[hh][i] = (iy0 << 16) | (ix0 & 0xffff);
        xrow[hh][i] = p.x + (((long)bt * p.H + oy * p.stride - p.pad) * p.W + ix0) * p.Cin;
      } else {
        xrow[hh][i] = p.x + (long)mm * p.ldx;
      }
    }
#pragma unroll
    for (int hh = 0; hh < WR; ++hh) {
      const int n = n0 + hh * 128 + wr_of(i);
      wok[hh][i] = n < p.N;
      wrow[hh][i] = p.w + (long)(wok[hh][i] ? n : 0) * p.K;
    }
  }
  const void* zero = (const void*)g_zero_page;
  // conv: when Cin % 64 == 0 a K tile never straddles a tap, so the tap is wave-uniform (scalar
  // math) and a lane only adds a scalar offset to its window base; otherwise per-lane division.
  // Each X quarter is staged for K tiles 0, 1, 2, ... in order, so its tap (ky, kx) and window
  // offset advance incrementally (no per-tile division): +BK channels, +(W - ks) * Cin on a row wrap.
  const bool tap_uniform = CONV && (p.Cin % BK == 0);
  int t_ci[2] = {0, 0}, t_kx[2] = {0, 0}, t_ky[2] = {0, 0};
  long t_off[2] = {0, 0};
  auto dma_x = [&](int kt, int buf, int i) {
    const int k0 = kt * BK;
    const int ky = t_ky[i], kx = t_kx[i];
    const long toff = t_off[i];
    if (tap_uniform) {
      t_off[i] += BK;
      t_ci[i] += BK;
      if (t_ci[i] == p.Cin) {
        t_ci[i] = 0;
        if (++t_kx[i] == p.ks) { t_kx[i] = 0; ++t_ky[i]; t_off[i] += (long)(p.W - p.ks) * p.Cin; }
      }
    }
#pragma unroll
    for (int hh = 0; hh < XR; ++hh) {
        const int k = k0 + kch0;
        const void* src = zero;
        if constexpr (CONV) {
          if (k < p.K) {
            if (tap_uniform) {
              if ((unsigned)((cyx[hh][i] >> 16) + ky) < (unsigned)p.H &&
                  (unsigned)((short)(cyx[hh][i] & 0xffff) + kx) < (unsigned)p.W)
                src = xrow[hh][i] + toff + kch0;
            } else {
              const int tap = k / p.Cin, ci = k - tap * p.Cin;
              const int ty = tap / p.ks, tx = tap - ty * p.ks;
              if ((unsigned)((cyx[hh][i] >> 16) + ty) < (unsigned)p.H &&
                  (unsigned)((short)(cyx[hh][i] & 0xffff) + tx) < (unsigned)p.W)
                src = xrow[hh][i] + ((long)ty * p.W + tx) * p.Cin + ci;
            }
          }
        } else if (xok[hh][i] && k < p.K) {
          src = xrow[hh][i] + k;
        }
        glds16(src, smem + buf * BUF + hh * HALF + (xr_of(i) - (lane >> 3)) * BK);
    }
  };
  auto dma_w = [&](int kt, int buf, int i) {
    const int k0 = kt * BK;
#pragma unroll
    for (int hh = 0; hh < WR; ++hh) {
      const int k = k0 + kch0;
      const void* src = (wok[hh][i] && k < p.K) ? (const void*)(wrow[hh][i] + k) : zero;
      glds16(src, smem + buf * BUF + (XR + hh) * HALF + (wr_of(i) - (lane >> 3)) * BK);
    }
  };
  // Dense GEMMs (K % 64 == 0, operands < 4 GiB): buffer_load ... lds with a per-lane byte offset
  // that never changes (row, chunk) and the K advance in the scalar soffset, so issuing a piece
  // costs no VALU at all; rows >= M / N get an offset past num_records and read zeros.
  __amdgpu_buffer_rsrc_t xrs, wrs;
  unsigned xvo[XR][2], wvo[WR][2];
  auto dense_offsets = [&](int m0_, int n0_, unsigned (&xv)[XR][2], unsigned (&wv)[WR][2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int hh = 0; hh < XR; ++hh) {
        const int m = m0_ + hh * 128 + xr_of(i);
        xv[hh][i] = m < p.M ? (unsigned)(((long)m * p.ldx + kch0) * 2) : 0x80000000u;
      }
#pragma unroll
      for (int hh = 0; hh < WR; ++hh) {
        const int n = n0_ + hh * 128 + wr_of(i);
        wv[hh][i] = n < p.N ? (unsigned)(((long)n * p.K + kch0) * 2) : 0x80000000u;
      }
    }
  };
  if constexpr (!CONV) {
    xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)(unsigned)((long)p.M * p.ldx * 2), 0x00020000);
    wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)(unsigned)((long)p.N * p.K * 2), 0x00020000);
    dense_offsets(m0, n0, xvo, wvo);
  }
  auto bdma_x = [&](int kt, int buf, int i, const unsigned (&xv)[XR][2]) {
#pragma unroll
    for (int hh = 0; hh < XR; ++hh)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (VDA_LDS void*)(smem + buf * BUF + hh * HALF + (xr_of(i) - (lane >> 3)) * BK),
                                               16, (int)xv[hh][i], kt * BK * 2, 0, 0);
  };
  auto bdma_w = [&](int kt, int buf, int i, const unsigned (&wv)[WR][2]) {
#pragma unroll
    for (int hh = 0; hh < WR; ++hh)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (VDA_LDS void*)(smem + buf * BUF + (XR + hh) * HALF + (wr_of(i) - (lane >> 3)) * BK),
                                               16, (int)wv[hh][i], kt * BK * 2, 0, 0);
  };
  auto stage_x = [&](int kt, int buf, int i) { if constexpr (CONV) dma_x(kt, buf, i); else bdma_x(kt, buf, i, xvo); };
  auto stage_w = [&](int kt, int buf, int i) { if constexpr (CONV) dma_w(kt, buf, i); else bdma_w(kt, buf, i, wvo); };

  f4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  // the next tile's prologue, issued by a chaining epilogue: K tile 0 (and the two K-tile-1 quarters
  // the 4-phase loop expects from "tile -1")
  auto chain_dma = [&](const unsigned (&xn)[XR][2], const unsigned (&wn2)[WR][2]) {
    bdma_x(0, 0, 0, xn); bdma_x(0, 0, 1, xn); bdma_w(0, 0, 0, wn2); bdma_w(0, 0, 1, wn2);
    if (nk > 1) { bdma_x(1, 1, 0, xn); bdma_w(1, 1, 1, wn2); }
  };
  const int frow = lane & 15, fchunk = lane >> 4;
  const bool prerelu = CONV && p.pre_relu;
  // wave's regions: X half wm (rows 0..127 of it), W half wn>>1 at row offset (wn&1)*64
  const int xoff = wm * HALF;
  const int woff = XR * HALF + (wn >> 1) * HALF;
  const int wrow0 = (wn & 1) * 64;

  // prologue: [Phi table,] all of tile 0, then the two tile-1 quarters the loop expects from "tile -1"
  // EK 3: the tile's (at most two) per-frame row-bias rows, 256 fp32 channels each, after the
  // statistics, in two slots by the parity of the block's tile index (a chaining epilogue stages the
  // next tile's rows while it still reads its own)
  float* rb_lds = reinterpret_cast<float*>(lnst_lds + 4096 + 1024);
  auto lnst_dma = [&](int m0_, int n0_, int vb_) {
    if constexpr (EK == 3) {
      if (wave < 2) {  // row 0 = the frame of tile row 0, row 1 = the next frame (rdiv >= 256: <= 2 per tile)
        const int rd = p.epi.rdiv;
        const int mrow = wave == 0 ? m0_ : min(m0_ + rd - m0_ % rd, p.M - 1);
        const int t = (mrow / rd) % p.epi.rmod;
        glds16(p.epi.rowbias + (long)t * p.N + n0_ + lane * 4,
               reinterpret_cast<h16*>(rb_lds + ((vb_ / (int)gridDim.x) & 1) * 512) + wave * 512);
      }
    }
    if constexpr (LNF) {
      if (p.epi.ln_parts <= 0) {  // rows m0 .. m0+255 of [M, 2] fp32 (mean, rstd): 2 pieces of 128 rows, waves 0-1
        if (wave < 2) {
          const int r = m0_ + wave * 128 + lane * 2;  // this lane's 16 B = rows r, r + 1
          // M odd: the piece of row M - 1 alone is read 8 B early (rows M - 2, M - 1), never past the
          // [M, 2] buffer; the readers find that row 8 B further on (lnst_ofs)
          const long f = (long)r * 2 - (r == p.M - 1 ? 2 : 0);
          const void* src = r < p.M ? (const void*)(p.epi.ln_stats + f) : (const void*)g_zero_page;
          glds16(src, lnst_lds + wave * 512);
        }
      } else if (wave < 2 * p.epi.ln_parts) {  // rows m0 .. m0+255 of [M, P, 2] partial sums: 2P pieces of 1 KiB
        const long f = (long)m0_ * p.epi.ln_parts * 2 + wave * 256 + lane * 4;  // float index of this lane's 16 B
        const long T = (long)p.M * p.epi.ln_parts * 2;
        // M * P odd: the last piece holds one valid entry; it is read 8 B early instead of 8 B past the end
        const void* src = f < T ? (const void*)(p.epi.ln_stats + (f + 4 > T ? f - 2 : f)) : (const void*)g_zero_page;
        glds16(src, lnst_lds + wave * 512);
      }
    }
  };
  constexpr int NIT_EPI = phased_nit<XR, WR, ACT>();
  if (!pre) {
    if constexpr (TAB) {
      const char* src = reinterpret_cast<const char*>(g_phi_tab) + tid * 16;
      glds16(src, smem + 2 * BUF + wave * 512);
      glds16(src + 8192, smem + 2 * BUF + 4096 + wave * 512);
    }
    lnst_dma(m0, n0, vb);
    TS(1);
    stage_x(0, 0, 0); stage_x(0, 0, 1); stage_w(0, 0, 0); stage_w(0, 0, 1);
    if (nk > 1) {
      stage_x(1, 1, 0); stage_w(1, 1, 1);
      wait_vmcnt<XR + WR>();
    } else {
      wait_vmcnt<0>();
    }
  } else {
    // issued by the previous tile's epilogue, followed by at least NIT_EPI output stores
    if (nk > 1) wait_vmcnt<XR + WR + NIT_EPI>();
    else wait_vmcnt<NIT_EPI>();
  }
  __builtin_amdgcn_s_barrier();
  TS(2);
  // LNF: the tile's 256 (mean, rstd) pairs are formed ONCE here, one row per thread of waves 0-3, from
  // the statistics the prologue staged (the producer's [M, P, 2] partial sums, or [M, 2] as is) into a
  // 2-KiB [256][2] table the epilogue reads after the main loop's barriers: the epilogue's lanes no
  // longer each reduce the partials of their 8 rows (4 lanes x 4 waves per row), and the staged
  // statistics are free for the next tile's prologue DMA as soon as this pass has read them.
  // The reads and the write go through asm: hipcc would put a vmcnt(0) before any LDS access here (a
  // pending LDS-DMA may alias it), draining the previous tile's output stores at every tile start.  The
  // statistics were retired by the prologue wait above and published by its barrier.
  float* lnfin = reinterpret_cast<float*>(lnst_lds + 4096);
  if constexpr (LNF && (EK == 1 || EK == 3)) {  // the register epilogues (the staged one reduces per row itself)
    if (tid < 256) {
      const float* st = reinterpret_cast<const float*>(lnst_lds);
      const int P = p.epi.ln_parts;
      const int sh = tid == lnst_shift_row(m0) ? 2 : 0;
      float2 mr;
      if (P <= 0) {
        mr = lds_ld_f2(st + 2 * tid + sh);
      } else {
        float sm = 0.f, sq = 0.f;
        if (P == 4) {  // the encoder's 1024 channels: the row's 4 partials as two 16-B reads (P even: no shift)
          float4 a, b;
          lds_ld_f4x2(st + 8 * tid, a, b);
          sm = ((a.x + a.z) + b.x) + b.z;
          sq = ((a.y + a.w) + b.y) + b.w;
        } else {
          for (int t = 0; t < P; ++t) {
            const float2 pq = lds_ld_f2(st + 2 * (tid * P + t) + (t == P - 1 ? sh : 0));
            sm += pq.x;
            sq += pq.y;
          }
        }
        const float invK = 1.f / (float)p.K;
        const float mean = sm * invK;
        mr = make_float2(mean, rsqrtf(fmaxf(fmaf(-mean, mean, sq * invK), 0.f) + p.epi.ln_eps));
      }
      lds_st_f2(lnfin + 2 * tid, mr);
    }
  }
  // Dense GEMMs: the epilogue's per-channel bias / gamma are fetched now, under the main loop,
  // instead of costing a dependent L2/MALL round trip after it (convs: no VGPR room, loaded later).
  constexpr bool PREF = !CONV && !ROWB;
  f4 pbv[4], pgv[4];
  if constexpr (PREF) {
    const vda_epilogue& e = p.epi;
    const int nq0 = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + wn * 64 + i * 16 + nq0;
      const int nc = n < p.N ? n : 0;
      pbv[i] = f4{0.f, 0.f, 0.f, 0.f};
      pgv[i] = f4{1.f, 1.f, 1.f, 1.f};
      if (has_bias) pbv[i] = *reinterpret_cast<const f4*>(e.bias + (ACT == VDA_ACT_GEGLU ? (n0 + wn * 64 + (i & ~1) * 16 + nq0 < p.N ? n0 + wn * 64 + (i & ~1) * 16 + nq0 : 0) + (i & 1) * 16 : nc));
      if constexpr (LNF) {
        pgv[i] = *reinterpret_cast<const f4*>(e.ln_colsum + nc);  // sum_k W[n, k] (LN fold)
      } else if (has_gamma) {
        if constexpr (ACT == VDA_ACT_GEGLU) {
          if (i % 2 == 0) pgv[i] = *reinterpret_cast<const f4*>(e.gamma + (n < p.N ? (n0 >> 1) + ((wn * 64 + i * 16) >> 1) + nq0 : 0));
        } else {
          pgv[i] = *reinterpret_cast<const f4*>(e.gamma + nc);
        }
      }
    }
  }
  const bool lagging = wave >= 4;
  if (lagging) __builtin_amdgcn_s_barrier();  // stagger waves 4-7 by one barrier

  h8 xf[4][2], wf[2][2];
  auto load_x = [&](const h16* base, int qm) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        xf[j][ks] = *reinterpret_cast<const h8*>(&base[xoff + swz(qm * 64 + j * 16 + frow, ks * 4 + fchunk)]);
        if (prerelu) xf[j][ks] = relu8(xf[j][ks]);
      }
  };
  auto load_w = [&](const h16* base, int qn) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        wf[i][ks] = *reinterpret_cast<const h8*>(&base[woff + swz(wrow0 + qn * 32 + i * 16 + frow, ks * 4 + fchunk)]);
  };
  auto mma = [&](int qm, int qn) {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[qn * 2 + i][qm * 4 + j] = mfma16(wf[i][ks], xf[j][ks], acc[qn * 2 + i][qm * 4 + j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  };

  unsigned tk = 0;  // dynamic schedule: the ticket in flight (wave 0, lane 0)
  // One quarter is staged per phase, each >= 2 phases after its last read (WAR under the stagger)
  // and retired by the P4 wait one phase before its first read:
  //   P1: Xq1(t+1) -> other buffer   P2: Wq0(t+1) -> other   P3: Xq0(t+2) -> this   P4: Wq1(t+2) -> this
  for (int kt = 0; kt < nk; ++kt) {
    const int cb = kt & 1, nb = cb ^ 1;
    const h16* base = smem + cb * BUF;
    const bool more1 = kt + 1 < nk, more2 = kt + 2 < nk;
    // P1
    load_x(base, 0);
    load_w(base, 0);
    if (more1) stage_x(kt + 1, nb, 1);
    mma(0, 0);
    // P2
    load_w(base, 1);
    if (more1) stage_w(kt + 1, nb, 0);
    mma(0, 1);
    // P3 (dynamic schedule: wave 0 draws the successor's ticket here, ahead of the quarters the P4 wait
    // leaves in flight, so that wait retires it)
    load_x(base, 1);
    if (tctr != nullptr && wave == 0 && kt == 0) {
      if (lane == 0) tk = ticket_draw(tctr);
    }
    if (more2) stage_x(kt + 2, cb, 0);
    mma(1, 1);
    // P4: retire everything but this tile's two P3/P4 quarters
    load_w(base, 0);
    if (more2) {
      stage_w(kt + 2, cb, 1);
      wait_vmcnt<XR + WR>();
    } else {
      wait_vmcnt<0>();
    }
    if (tctr != nullptr && wave == 0 && kt == 0) {  // the draw has landed: publish the successor
      if (lane == 0) ticket_publish(tslot, tk, tbase);
    }
    mma(1, 0);
  }
  if (!lagging) __builtin_amdgcn_s_barrier();  // balance the stagger
  TS(3);
  // the successor: published by wave 0 before step 0's last barrier (retired by the lgkmcnt waits after it)
  int succ = vb_next;
  if (tctr != nullptr) {
    succ = __builtin_amdgcn_readfirstlane(lds_ld_i1(tslot));
    if (succ >= tiles_m * tiles_n) succ = -1;
  }
  vb_next = EK != 0 ? succ : -1;  // the chained prologue

  const int mcol = lane & 15, nq = (lane >> 4) * 4;
  if constexpr ((EK == 1 || EK == 3) && XR == 2 && WR == 2) {
    // Register epilogue (qkv, fc1): no LDS staging.  The LN statistics of the lane's 8 rows come out of
    // LDS first; then one barrier frees the operand buffers and the next tile's prologue DMA goes out
    // at once, landing under this tile's activation work and stores.  Pairs of accumulators (channels
    // 16i.. and 16(i+1)..) are exchanged across 16-lane rows with v_permlane16_swap, after which every
    // lane holds 8 consecutive channels of its row; a DPP row_ror:8 exchange between lanes l and l ^ 8
    // then lets each 16-byte-per-lane store write 8 whole 128-B lines.  EK 3 (the motion-module q/k/v)
    // adds the row's frame PE row bias from the two rows staged in LDS.
    const vda_epilogue& e = p.epi;
    const int rbslot = (vb / (int)gridDim.x) & 1;
    const int rbnd = EK == 3 ? e.rdiv - m0 % e.rdiv : 0;  // first tile row of the next frame
    // The row statistics (lnfin) and the prefetched bias / colsum are taken into registers BEFORE the
    // next tile's prologue DMA goes out: hipcc waits vmcnt(0) at their first use, which is free here
    // and would drain that DMA after it.
    float2 mr[8];
    if constexpr (LNF) {
#pragma unroll
      for (int j = 0; j < 8; ++j) mr[j] = *reinterpret_cast<const float2*>(lnfin + 2 * (wm * 128 + j * 16 + mcol));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(pbv[i]), "v"(pgv[i]));
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's statistics reads have landed
    // every LDS operand read of this tile is done (its MFMAs consumed them): hand the operand buffers
    // and the staged statistics (already reduced into lnfin) to the next tile's prologue DMA
    __builtin_amdgcn_s_barrier();
    if constexpr (!CONV) {
      if (vb_next >= 0) {
        int tmn, tnn;
        tile_coords(vb_next, tiles_m * tiles_n, tiles_m, tiles_n, tmn, tnn);
        unsigned xn[XR][2], wn2[WR][2];
        dense_offsets(tmn * BM, tnn * BN, xn, wn2);
        lnst_dma(tmn * BM, tnn * BN, vb_next);
        chain_dma(xn, wn2);
      }
    }
    TS(4);
    static_assert(phased_nit<XR, WR, ACT>() == 16, "the register epilogue issues 16 stores per lane");
    const int g = lane >> 4;
    // row drop (vda_epilogue.drop_period, the projects GEMM on a tap with the cls rows left out): source
    // row m0 + r of frame f goes to Y row m0 + r - f - 1, the frame's first row nowhere.  drop_period >= 256,
    // so a tile meets at most one frame boundary (tile row rbd).  Y base row ybase = Y row of m0 (or 0).
    const int dp = e.drop_period;
    const int f0 = dp > 0 ? m0 / dp : 0;
    const int rbd = dp > 0 ? (f0 + 1) * dp - m0 : 1 << 30;
    const bool cls0 = dp > 0 && m0 % dp == 0;
    const long ybase = dp > 0 ? (m0 - f0 - (cls0 ? 0 : 1)) : m0;
    const long yrows = dp > 0 ? (long)p.M - (p.M + dp - 1) / dp : p.M;
    const long mrows = yrows - ybase;
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.y + ybase * p.ldy), (short)0,
        (int)(mrows * p.ldy * 2 < 0x7fffffffL ? mrows * p.ldy * 2 : 0x7fffffffL), 0x00020000);
    // byte offset of tile row r in ry (0x80000000: not stored)
    auto yrow = [&](int r) -> unsigned {
      if (dp == 0) return (unsigned)(r * p.ldy * 2);
      if ((cls0 && r == 0) || r == rbd) return 0x80000000u;
      return (unsigned)((m0 + r - f0 - (r > rbd ? 2 : 1) - ybase) * p.ldy * 2);
    };
    unsigned cofs[2];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int col = n0 + wn * 64 + 32 * pp + 16 * (g & 1) + 8 * (g >> 1);
      cofs[pp] = col < p.N ? (unsigned)(col * 2) : 0x80000000u;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = acc[i][j];
        if constexpr (LNF) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[i][r] = fmaf(mr[j].y, fmaf(-mr[j].x, pgv[i][r], v[i][r]), pbv[i][r]);
        } else {
          v[i] += pbv[i];
        }
        if constexpr (EK == 3) {  // + the row's frame PE row bias (slot row 1 past the frame boundary)
          const int rl = wm * 128 + j * 16 + mcol;
          v[i] += *reinterpret_cast<const f4*>(rb_lds + rbslot * 512 + (rl >= rbnd ? 256 : 0) + wn * 64 + i * 16 + nq);
        }
        if constexpr (ACT == VDA_ACT_GELU && !TAB) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[i][r] = gelu_erf(v[i][r]);
        }
      }
      if constexpr (ACT == VDA_ACT_GELU && TAB) {
        // the row's 16 table lines are all requested before the first is used (one LDS round trip per
        // row instead of a wait per group of reads)
        phi_f2 ab[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) ab[k] = phi_line(v[k / 4][k % 4], phib);
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k / 4][k % 4] *= fmaf(v[k / 4][k % 4], ab[k].y, ab[k].x);
      }
      u32x4 o[2];
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        float a[4], c[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          a[r] = v[2 * pp][r];
          c[r] = v[2 * pp + 1][r];
          perm16_swap(a[r], c[r]);
        }
        typedef float f2v __attribute__((ext_vector_type(2)));
        const h2 h0 = __builtin_convertvector(f2v{a[0], a[1]}, h2), h1 = __builtin_convertvector(f2v{a[2], a[3]}, h2);
        const h2 h2_ = __builtin_convertvector(f2v{c[0], c[1]}, h2), h3 = __builtin_convertvector(f2v{c[2], c[3]}, h2);
        o[pp] = u32x4{__builtin_bit_cast(unsigned, h0), __builtin_bit_cast(unsigned, h1),
                      __builtin_bit_cast(unsigned, h2_), __builtin_bit_cast(unsigned, h3)};
      }
      // whole 128-B lines per store: lanes mcol < 8 trade their pp = 1 piece for the pp = 0 piece of
      // row mcol + 8 (DPP row_ror:8 swaps lanes l and l ^ 8 of each 16-lane row), so one store covers
      // rows mcol & 7 (A) and the other rows 8 + (mcol & 7) (B), each row's 64 channels in one go
      // (64-B half lines measured 430 MB of WRITE_SIZE for fc1's 359 MB of output)
      const bool lo8 = (mcol & 8) == 0;
      u32x4 A, B;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned snd = lo8 ? o[1][k] : o[0][k];
        const unsigned got = (unsigned)__builtin_amdgcn_mov_dpp((int)snd, 0x128, 0xF, 0xF, true);
        A[k] = lo8 ? o[0][k] : got;
        B[k] = lo8 ? got : o[1][k];
      }
      const int ra = wm * 128 + j * 16 + (mcol & 7);
      const unsigned co = lo8 ? cofs[0] : cofs[1];  // N % 256 == 0 with drop_period: never the sentinel
      const unsigned ya = yrow(ra), yb = yrow(ra + 8);
      const unsigned rA = ya == 0x80000000u ? ya : ya + co;
      const unsigned rB = yb == 0x80000000u ? yb : yb + co;
      __builtin_amdgcn_raw_buffer_store_b128(A, ry, rA, 0, VDA_EPI_STORE_AUX);
      __builtin_amdgcn_raw_buffer_store_b128(B, ry, rB, 0, VDA_EPI_STORE_AUX);
    }
    TS(5);
    return succ;
  }
  if constexpr (EK == 2 && XR == 2 && WR == 2) {
    // Register epilogue with one residual and the row statistics (proj, fc2: x += ...): the residual
    // rows are requested first (in the whole-line layout the stores use, below), then the operand
    // buffers are handed to the next tile's prologue DMA as above.  Output =
    // fp16(acc + bias) + residual in packed fp16, as the staged epilogue.  Row statistics: (sum, sumsq)
    // of the stored fp16 values per lane, over the 4 lanes of a row by permlane swaps, over the 4 waves
    // of a 256-column block through an 8-KiB LDS table.
    const vda_epilogue& e = p.epi;
    const int g = lane >> 4;
    const long mrows = p.M - m0;
    auto rsrc_rows = [&](const void* base, long ld) {
      return __builtin_amdgcn_make_buffer_rsrc((void*)((const h16*)base + (long)m0 * ld), (short)0,
                                               (int)(mrows * ld * 2 < 0x7fffffffL ? mrows * ld * 2 : 0x7fffffffL), 0x00020000);
    };
    int ccol[2];
    bool cok[2];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      ccol[pp] = n0 + wn * 64 + 32 * pp + 16 * (g & 1) + 8 * (g >> 1);
      cok[pp] = ccol[pp] < p.N;
    }
    // Whole 128-B lines, as the EK 1 epilogue: after the permlane swap a lane holds 8 consecutive
    // channels of its row mcol; a DPP row_ror:8 exchange between lanes l and l ^ 8 then gives every lane
    // 8 channels of row mcol & 7 (A) and of row 8 + (mcol & 7) (B) at one column offset, so each 16-B
    // store (and each residual load, requested in that layout up front) covers whole lines.
    const bool lo8 = (mcol & 8) == 0;
    const int colx = lo8 ? ccol[0] : ccol[1];
    const bool cokx = lo8 ? cok[0] : cok[1];
    const __amdgpu_buffer_rsrc_t rr = rsrc_rows(e.res, e.ldres);
    h8 rv[8][2];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int ab = 0; ab < 2; ++ab) {
        const long row = wm * 128 + j * 16 + (mcol & 7) + 8 * ab;
        const unsigned o = cokx ? (unsigned)((row * e.ldres + colx) * 2) : 0x80000000u;
        rv[j][ab] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rr, o, 0, 0));
      }
    __builtin_amdgcn_s_barrier();  // every wave is done reading the operand buffers
    if constexpr (!CONV) {
      if (vb_next >= 0) {
        int tmn, tnn;
        tile_coords(vb_next, tiles_m * tiles_n, tiles_m, tiles_n, tmn, tnn);
        unsigned xn[XR][2], wn2[WR][2];
        dense_offsets(tmn * BM, tnn * BN, xn, wn2);
        chain_dma(xn, wn2);
      }
    }
    static_assert(phased_nit<XR, WR, ACT>() == 16, "the register epilogue issues 16 stores per lane");
    const __amdgpu_buffer_rsrc_t ry = rsrc_rows(p.y, p.ldy);
    float* red = reinterpret_cast<float*>(smem + 2 * BUF);  // [4 wn][256 rows][2]
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int rl = wm * 128 + j * 16 + mcol;
      u32x4 o[2];
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        float a[4], c[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          a[r] = acc[2 * pp][j][r] + pbv[2 * pp][r];
          c[r] = acc[2 * pp + 1][j][r] + pbv[2 * pp + 1][r];
          perm16_swap(a[r], c[r]);
        }
        typedef float f2v __attribute__((ext_vector_type(2)));
        const h2 h0 = __builtin_convertvector(f2v{a[0], a[1]}, h2), h1 = __builtin_convertvector(f2v{a[2], a[3]}, h2);
        const h2 h2_ = __builtin_convertvector(f2v{c[0], c[1]}, h2), h3 = __builtin_convertvector(f2v{c[2], c[3]}, h2);
        o[pp] = u32x4{__builtin_bit_cast(unsigned, h0), __builtin_bit_cast(unsigned, h1),
                      __builtin_bit_cast(unsigned, h2_), __builtin_bit_cast(unsigned, h3)};
      }
      u32x4 A, B;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned snd = lo8 ? o[1][k] : o[0][k];
        const unsigned got = (unsigned)__builtin_amdgcn_mov_dpp((int)snd, 0x128, 0xF, 0xF, true);
        A[k] = lo8 ? o[0][k] : got;
        B[k] = lo8 ? got : o[1][k];
      }
      const h8 tA = __builtin_bit_cast(h8, A) + rv[j][0];
      const h8 tB = __builtin_bit_cast(h8, B) + rv[j][1];
      const unsigned rA = cokx ? (unsigned)(((long)(wm * 128 + j * 16 + (mcol & 7)) * p.ldy + colx) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, tA), ry, rA, 0, VDA_EPI_STORE_AUX);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, tB), ry, rA + (unsigned)(8 * p.ldy * 2), 0,
                                             VDA_EPI_STORE_AUX);
      float sA, qA, sB, qB;
      stat_acc(cokx ? tA : h8{0, 0, 0, 0, 0, 0, 0, 0}, sA, qA);
      stat_acc(cokx ? tB : h8{0, 0, 0, 0, 0, 0, 0, 0}, sB, qB);
      // lane l keeps row mcol (l < 8 of its 16: A, else B) and adds its partner l ^ 8's piece of that row
      float ssum = (lo8 ? sA : sB) + dpp_f<0x128>(lo8 ? sB : sA);
      float ssq = (lo8 ? qA : qB) + dpp_f<0x128>(lo8 ? qB : qA);
      // the row's 64 channels of this wave sit in lanes mcol, mcol + 16, + 32, + 48
      float x0, x1;
      swap16_pair(ssum, x0, x1); ssum = x0 + x1;
      swap16_pair(ssq, x0, x1); ssq = x0 + x1;
      swap32_pair(ssum, x0, x1); ssum = x0 + x1;
      swap32_pair(ssq, x0, x1); ssq = x0 + x1;
      if (g == 0) lds_st_f2(red + 2 * (wn * 256 + rl), make_float2(ssum, ssq));  // asm: no LDS-DMA vmcnt
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    {  // thread -> (row, statistic): the 4 column-slices of the 256-column block, in a fixed order
      const int row = tid >> 1, st = tid & 1;
      const float v = lds_ld_f1(red + 2 * row + st) + lds_ld_f1(red + 2 * (256 + row) + st) +
                      lds_ld_f1(red + 2 * (512 + row) + st) + lds_ld_f1(red + 2 * (768 + row) + st);
      const int P = (p.N + 255) / 256;
      const int m = m0 + row;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)e.stats_out, (short)0, (int)((long)p.M * P * 8), 0x00020000);
      const unsigned vo = m < p.M ? (unsigned)((((long)m * P + (n0 >> 8)) * 2 + st) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rs, vo, 0, 0);
    }
    TS(5);
    return succ;
  }
  if (rows_store) {
    // LDS-staged epilogue: phase 1 writes t = gamma * act(acc + bias + rowbias) as fp16 into a
    // [256][OW] image (8-byte units XOR-swizzled by row&15: conflict-free both ways); phase 2 reads
    // it back as whole rows, adds the residual(s) with 16-byte loads and stores 16-byte chunks, so
    // every output row is written by full contiguous 128-B lines.
    constexpr int OW = (ACT == VDA_ACT_GEGLU) ? BN / 2 : BN;  // output columns of this tile
    __syncthreads();                                         // all waves done with the operand image
    const vda_epilogue& e = p.epi;
    // Per-channel operands are loaded ONCE per lane, unconditionally from clamped addresses, before
    // any math: a load under a per-element condition makes hipcc branch around it and wait for
    // each one in turn (32 dependent L2 round trips per tile).
    bool nok[4];
    int ncl[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + wn * 64 + i * 16 + nq;
      nok[i] = n < p.N;
      ncl[i] = nok[i] ? n : 0;
    }
    if constexpr (LNF) {  // y = rstd * (acc - mean * colsum) + bias (LayerNorm folded, before the activation)
      const float* st = reinterpret_cast<const float*>(lnst_lds);
      const f4* bv = pbv;  // zero when there is no bias
      const int P = e.ln_parts;
      const float invK = 1.f / (float)p.K;
      const int srow = lnst_shift_row(m0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int rl = wm * 128 + j * 16 + mcol;
        const int sh = rl == srow ? 2 : 0;
        float2 mr;
        if (P <= 0) {
          mr = *reinterpret_cast<const float2*>(st + 2 * rl + sh);
        } else {  // partial (sum, sumsq) of P column blocks -> (mean, rstd)
          float sm = 0.f, sq = 0.f;
          for (int t = 0; t < P; ++t) {
            const float2 pq = *reinterpret_cast<const float2*>(st + 2 * (rl * P + t) + (t == P - 1 ? sh : 0));
            sm += pq.x;
            sq += pq.y;
          }
          const float mean = sm * invK;
          const float var = fmaxf(fmaf(-mean, mean, sq * invK), 0.f);
          mr = make_float2(mean, rsqrtf(var + e.ln_eps));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc[i][j][r] = fmaf(mr.y, fmaf(-mr.x, pgv[i][r], acc[i][j][r]), bv[i][r]);
      }
    } else if (has_bias) {  // bias folded into the accumulators up front (GEGLU: h and g halves alike)
      f4 bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        bv[i] = PREF ? pbv[i] : *reinterpret_cast<const f4*>(e.bias + (ACT == VDA_ACT_GEGLU ? ncl[i & ~1] + (i & 1) * 16 : ncl[i]));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] += bv[i];
    }
    if constexpr (ACT != VDA_ACT_GEGLU && ROWB) {
      if (e.rowbias) {  // per-row bias (folded positional terms): 4 loads per output row group
        // (m / rdiv) % rmod by fp32 reciprocals + one integer correction each (m < 2^24: exact)
        const float inv_div = 1.f / (float)e.rdiv, inv_mod = 1.f / (float)e.rmod;
        // RBD row groups in flight: the row-bias table (the patch embed's 5.6 MB) is not L2-resident,
        // so one group at a time pays 8 MALL round trips per tile
        auto rb_load = [&](int j, f4 (&rb)[4]) {
          const int m = m0 + wm * 128 + j * 16 + mcol;
          int qd = (int)((float)m * inv_div);
          qd += (m - qd * e.rdiv >= e.rdiv) ? 1 : 0;
          qd -= (m < qd * e.rdiv) ? 1 : 0;
          int qm = (int)((float)qd * inv_mod);
          qm += (qd - qm * e.rmod >= e.rmod) ? 1 : 0;
          qm -= (qd < qm * e.rmod) ? 1 : 0;
          const long roff = m < p.M ? (long)(qd - qm * e.rmod) * p.N : 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) rb[i] = *reinterpret_cast<const f4*>(e.rowbias + roff + ncl[i]);
        };
        constexpr int RBD = 2;  // tools/ab_gemm.py --shapes patch: 1: 97.2, 2: 91.8, 3: 97.5 us
        f4 rb[RBD][4];
#pragma unroll
        for (int j = 0; j < RBD - 1; ++j) rb_load(j, rb[j]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (j + RBD - 1 < 8) rb_load(j + RBD - 1, rb[(j + RBD - 1) % RBD]);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][j] += rb[j % RBD][i];
          __builtin_amdgcn_sched_barrier(0);  // keep the loads of row group j+RBD after these adds
        }
      }
    }
    // gamma (layer scale) is normally folded into W and b by the host; the multiply is compiled
    // only into the has-gamma variant of the loop, and fp32 -> fp16 goes through v_cvt_pk_f16_f32
    if constexpr (ACT == VDA_ACT_GELU && TAB) {
      // table GELU in place on the accumulators, 16 values per step: all 16 LDS reads are issued
      // before the first is consumed (one wait per group instead of one per value)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; j += 4) {
          phi_f2 ab[16];
#pragma unroll
          for (int k = 0; k < 16; ++k) ab[k] = phi_line(acc[i][j + k / 4][k % 4], phib);
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const float a = acc[i][j + k / 4][k % 4];
            acc[i][j + k / 4][k % 4] = a * fmaf(a, ab[k].y, ab[k].x);
          }
        }
    }
    if constexpr (ACT == VDA_ACT_GEGLU && TAB) {
      // the gate halves (accumulators 1 and 3) through the table GELU in place, 16 values per step with
      // all 16 LDS reads issued before the first is consumed (as the GELU pass above)
#pragma unroll
      for (int i = 1; i < 4; i += 2)
#pragma unroll
        for (int j = 0; j < 8; j += 4) {
          phi_f2 ab[16];
#pragma unroll
          for (int k = 0; k < 16; ++k) ab[k] = phi_line(acc[i][j + k / 4][k % 4], phib);
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const float a = acc[i][j + k / 4][k % 4];
            acc[i][j + k / 4][k % 4] = a * fmaf(a, ab[k].y, ab[k].x);
          }
        }
    }
    auto phase1 = [&](auto g_tag) {
      constexpr bool HG = decltype(g_tag)::value;
#pragma unroll
      for (int i = 0; i < 4; i += (ACT == VDA_ACT_GEGLU ? 2 : 1)) {
        const int nl = wn * 64 + i * 16 + nq;  // local W row of this lane's first channel
        f4 gv = f4{1.f, 1.f, 1.f, 1.f};
        if constexpr (HG) {
          if constexpr (PREF) gv = pgv[i];
          else gv = *reinterpret_cast<const f4*>(e.gamma + (ACT == VDA_ACT_GEGLU ? (nok[i] ? (n0 >> 1) + ((wn * 64 + i * 16) >> 1) + nq : 0) : ncl[i]));
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int ml = wm * 128 + j * 16 + mcol;
          f4 v;
          int col;
          if constexpr (ACT == VDA_ACT_GEGLU) {
            const f4 vh = acc[i][j], vg = acc[i + 1][j];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = vh[r] * (TAB ? vg[r] : gelu_erf(vg[r]));  // TAB: gate done above
            col = ((wn * 64 + i * 16) >> 1) + nq;
          } else {
            v = acc[i][j];
            if constexpr (ACT == VDA_ACT_GELU && !TAB) {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
            } else if constexpr (ACT == VDA_ACT_RELU) {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
            }
            col = nl;
          }
          if constexpr (HG) v *= gv;
          typedef float f2v __attribute__((ext_vector_type(2)));
          const h2 lo = __builtin_convertvector(f2v{v[0], v[1]}, h2);
          const h2 hi = __builtin_convertvector(f2v{v[2], v[3]}, h2);
          const int u = (col >> 2) ^ (ml & 15);
          *reinterpret_cast<uint2*>(&smem[ml * OW + u * 4]) = make_uint2(__builtin_bit_cast(unsigned, lo), __builtin_bit_cast(unsigned, hi));
        }
      }
    };
    const int nout = (ACT == VDA_ACT_GEGLU) ? (p.N >> 1) : p.N;
    const int cout0 = (ACT == VDA_ACT_GEGLU) ? (n0 >> 1) : n0;
    // Phase 2: thread -> fixed (row0 + RPI * it, 16-byte chunk q).  Every iteration reuses the same
    // LDS swizzle and advances both addresses by constants; stores (and residual loads) are buffer
    // ops whose range check drops rows >= M and chunks >= nout (offset 0x80000000), so the loop
    // has no branches and no per-iteration address math beyond one add.  Residuals are added in
    // packed fp16 (one rounding per add, as the reference's fp16 adds).
    constexpr int CPR = OW / 8;    // 16-byte chunks per row
    constexpr int RPI = 512 / CPR; // rows per iteration (a multiple of 16: the swizzle repeats)
    constexpr int NIT = BM / RPI;
    const int q = tid % CPR, row0 = tid / CPR;
    const int sw = row0 & 15;
    const h16* l0 = smem + row0 * OW + ((2 * q) ^ sw) * 4;
    const h16* l1 = smem + row0 * OW + ((2 * q + 1) ^ sw) * 4;
    const int c = cout0 + q * 8;
    const long mrows = p.M - m0;
    auto rsrc = [&](const h16* base, long ld) {
      return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (long)m0 * ld), (short)0,
                                               (int)(mrows * ld * 2 < 0x7fffffffL ? mrows * ld * 2 : 0x7fffffffL), 0x00020000);
    };
    auto voff = [&](long ld) { return c < nout ? (unsigned)(((long)row0 * ld + c) * 2) : 0x80000000u; };
    const __amdgpu_buffer_rsrc_t ry = rsrc(p.y, p.ldy);
    const unsigned vy = voff(p.ldy), sy = (unsigned)(RPI * p.ldy * 2);
    const h16* r1p = (const h16*)(has_res ? e.res : e.res2);
    const long r1ld = has_res ? e.ldres : e.ldres2;
    const int nres = (has_res ? 1 : 0) + (has_res2 ? 1 : 0);
    // A single residual (the encoder's proj / fc2 x += ..., the fusion adds) is requested in full
    // here, before phase 1, so its 16 loads per thread overlap the activation / LDS staging instead
    // of stalling phase 2 four times per tile (in situ, proj ran 45 % over its residual-free time).
    // The residual may alias the output: this tile is written only by this block, in phase 2.
    constexpr bool RPF = XR == 2 && ACT == VDA_ACT_NONE && !CONV && !ROWB && !LNF;  // NIT = 16 chunks = 64 VGPRs; the
    // other instantiations have no register room for it (GELU / GEGLU / conv / row bias: spills)
    h8 rpre[RPF ? NIT : 1];
    if constexpr (RPF) {
      if (nres == 1) {
        const __amdgpu_buffer_rsrc_t rr = rsrc(r1p, r1ld);
        const unsigned vr = voff(r1ld), sr = (unsigned)(RPI * r1ld * 2);
#pragma unroll
        for (int it = 0; it < NIT; ++it)
          rpre[it] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rr, vr + it * sr, 0, 0));
      }
    }
    if (!LNF && has_gamma) phase1(std::true_type{});
    else phase1(std::false_type{});
    __syncthreads();
    TS(4);
    // Phase 2a: the whole staged tile back into registers (the accumulators are dead by now), then,
    // for a persistent dense block with another tile to run, one barrier (every wave's reads have
    // landed) and the next tile's prologue DMA into the freed operand buffers, issued before this
    // tile's stores (see gemm256_tile's header).
    static_assert(NIT == NIT_EPI, "phased_nit() must match the phase-2 store count");
    h8 tv[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const uint2 lo = *reinterpret_cast<const uint2*>(l0 + it * RPI * OW);
      const uint2 hi = *reinterpret_cast<const uint2*>(l1 + it * RPI * OW);
      tv[it] = __builtin_bit_cast(h8, make_uint4(lo.x, lo.y, hi.x, hi.y));
    }
    if constexpr (!CONV) {
      if (vb_next >= 0) {
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's staged-tile reads are in registers
        __builtin_amdgcn_s_barrier();
        int tmn, tnn;
        tile_coords(vb_next, tiles_m * tiles_n, tiles_m, tiles_n, tmn, tnn);
        unsigned xn[XR][2], wn2[WR][2];
        dense_offsets(tmn * BM, tnn * BN, xn, wn2);
        lnst_dma(tmn * BM, tnn * BN, vb_next);
        chain_dma(xn, wn2);
      }
    }
    auto phase2 = [&](auto nres_tag) {
      constexpr int NR = decltype(nres_tag)::value;
      __amdgpu_buffer_rsrc_t rr1, rr2;
      unsigned vr1 = 0, sr1 = 0, vr2 = 0, sr2 = 0;
      if constexpr (NR >= 1) { rr1 = rsrc(r1p, r1ld); vr1 = voff(r1ld); sr1 = (unsigned)(RPI * r1ld * 2); }
      if constexpr (NR >= 2) { rr2 = rsrc((const h16*)e.res2, e.ldres2); vr2 = voff(e.ldres2); sr2 = (unsigned)(RPI * e.ldres2 * 2); }
      // residual loads run PD iterations ahead of their use (a rolling window instead of batches of
      // 4 loads whose latency each batch waits out)
      constexpr int PD = 4;
      h8 q1[PD], q2[PD];
      auto ld1 = [&](int it) { return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rr1, vr1 + it * sr1, 0, 0)); };
      auto ld2 = [&](int it) { return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rr2, vr2 + it * sr2, 0, 0)); };
#pragma unroll
      for (int it = 0; it < PD && it < NIT; ++it) {
        if constexpr (NR >= 1) q1[it] = ld1(it);
        if constexpr (NR >= 2) q2[it] = ld2(it);
      }
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        h8 t = tv[it];
        if constexpr (NR >= 1) {
          t += q1[it % PD];
          if (it + PD < NIT) q1[it % PD] = ld1(it + PD);
        }
        if constexpr (NR >= 2) {
          t += q2[it % PD];
          if (it + PD < NIT) q2[it % PD] = ld2(it + PD);
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, t), ry, vy + it * sy, 0, VDA_EPI_STORE_AUX);
      }
    };
    // + per-row partial (sum, sumsq) of the stored values for a following LN fold (the stored tile
    // values tv [+ the prefetched residual]): a half-wave per row, 16 rows per lane
    auto store_with_stats = [&](auto with_res) {
      constexpr bool WR1 = decltype(with_res)::value;
      static_assert(NIT == 16 && RPI == 16, "stats: a half-wave per row, 16 rows per lane");
      const bool cval = c < nout;
      float v[32];
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        h8 t = tv[it];
        if constexpr (WR1) t += rpre[it];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, t), ry, vy + it * sy, 0, VDA_EPI_STORE_AUX);
        stat_acc(cval ? t : h8{0, 0, 0, 0, 0, 0, 0, 0}, v[it], v[16 + it]);
      }
      const float r = halfwave_sum32(v, lane);
      const int P = (p.N + 255) / 256;
      const int m = m0 + row0 + 16 * (lane & 15);
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)e.stats_out, (short)0, (int)((long)p.M * P * 8), 0x00020000);
      const unsigned vo = m < p.M ? (unsigned)((((long)m * P + (n0 >> 8)) * 2 + ((lane >> 4) & 1)) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, r), rs, vo, 0, 0);
    };
    // pixel shuffle (ps_rows): tile row m = input pixel (bt, yh, xw), its 256 columns = channels co0 ..
    // co0 + 255 of output pixel (yh k + ki, xw k + kj); the row walk advances (xw, yh, bt) incrementally
    // (RPI = 16 rows per step, ps_win >= 16: at most one wrap)
    auto ps_store = [&]() {
      if constexpr (RPI == 16 && ACT != VDA_ACT_GEGLU && !ROWB && XR == 2) {  // the instantiations ps_rows admits
      const int k = e.ps_k, cout = e.ps_cout, win = e.ps_win, hin = e.ps_hin;
      const int ij = n0 / cout, co0 = n0 - ij * cout, ki = ij / k, kj = ij - ki * k;
      const __amdgpu_buffer_rsrc_t rz =
          __builtin_amdgcn_make_buffer_rsrc((void*)p.y, (short)0, (int)((long)p.M * p.N * 2), 0x00020000);
      int m = m0 + row0;
      int xw = m % win, tq = m / win;
      int yh = tq % hin, bt = tq / hin;
      const long rowlen = (long)win * k;
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const long pix = ((long)(bt * hin + yh) * k + ki) * rowlen + (long)xw * k + kj;
        const unsigned off = m < p.M ? (unsigned)((pix * cout + co0 + q * 8) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, tv[it]), rz, off, 0, VDA_EPI_STORE_AUX);
        m += RPI;
        xw += RPI;
        if (xw >= win) {
          xw -= win;
          if (++yh == hin) { yh = 0; ++bt; }
        }
      }
      }
    };
    if (ps_rows) {
      ps_store();
    } else if (nres == 0) {
      if constexpr (RPF) {
        if (has_stats) store_with_stats(std::false_type{});
        else phase2(std::integral_constant<int, 0>{});
      } else {
        phase2(std::integral_constant<int, 0>{});
      }
    } else if (nres == 1) {
      if constexpr (RPF) {
        if (has_stats) {
          store_with_stats(std::true_type{});
        } else {
#pragma unroll
          for (int it = 0; it < NIT; ++it) {
            const h8 t = tv[it] + rpre[it];
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, t), ry, vy + it * sy, 0, VDA_EPI_STORE_AUX);
          }
        }
      } else {
        phase2(std::integral_constant<int, 1>{});
      }
    } else {
      phase2(std::integral_constant<int, 2>{});
    }
    TS(5);
    return succ;
  }
  if constexpr (PREF) {  // unused here: retire the prefetch loads inside the tile (no load pending across tiles)
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(pbv[i]), "v"(pgv[i]));
  }
  if constexpr (EK != 0) {
    return succ;  // row store only
  } else if constexpr (ACT == VDA_ACT_GEGLU) {
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
      const int nbase = n0 + wn * 64 + i * 16;
      if (nbase >= p.N) continue;
      const int n_out = (nbase >> 1) + nq;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = m0 + wm * 128 + j * 16 + mcol;
        if (m < p.M) epi_geglu4(p, m, nbase + nq, nbase + 16 + nq, n_out, acc[i][j], acc[i + 1][j]);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + wn * 64 + i * 16 + nq;
      if (n >= p.N) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = m0 + wm * 128 + j * 16 + mcol;
        if (m < p.M) epi_store4<ACT>(p, m, n, acc[i][j]);
      }
    }
  }
  return succ;
}

// Persistent: one block per CU walks tiles vb, vb + gridDim.x, ... (virtual block ids keep the
// XCD-aware tile mapping of a one-tile-per-block grid).  All blocks run equal-length tiles, so left
// alone every CU would hit its epilogue (HBM store burst) and next prologue (load burst) at the same
// moment while the MFMAs idle.  When the last round is short (ntiles % grid <= grid / 2), half of
// the blocks that own one tile fewer start half a tile late (stagger_ticks of the 100 MHz
// s_memrealtime clock): the bursts of the two halves then overlap the other half's main loop, and
// the delayed blocks still finish no later than the blocks with the extra tile.
template <int XR, int WR, bool CONV, int ACT, bool ROWB, bool LNF = false, int EK = 0>
__global__ __launch_bounds__(512) void gemm256_kernel(GemmParams p, int tiles_m, int tiles_n, int stagger_ticks,
                                                      int desync) {
  constexpr int BUF = (XR + WR) * 128 * BK;
  constexpr bool TAB = XR == 2 && (ACT == VDA_ACT_GELU || ACT == VDA_ACT_GEGLU);
  // + 64 halves at the end (XR 2): the dynamic schedule's successor slot
  constexpr int SMEM_HALVES = 2 * BUF + (TAB ? PHI_LDS_HALVES : 0) + (LNF ? 4096 + 1024 : 0) + (EK == 2 ? 4096 : 0) +
                              (EK == 3 ? 2048 : 0) + (XR == 2 ? 64 : 0);
  __shared__ __attribute__((aligned(1024))) h16 smem[SMEM_HALVES];
  const int ntiles = tiles_m * tiles_n;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  if (desync > 1) {  // tuning experiment: every block starts ((b / 8) % desync) / desync of stagger_ticks late
    const uint64_t d = (uint64_t)(((blockIdx.x >> 3) % desync) * stagger_ticks / desync);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < d) __builtin_amdgcn_s_sleep(16);
  } else if (stagger_ticks > 0 && (int)blockIdx.x >= ntiles % (int)gridDim.x && ((blockIdx.x >> 3) & 1)) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)stagger_ticks) __builtin_amdgcn_s_sleep(16);
  }
  if constexpr (CONV) {  // convs launch one block per tile (phased_sched): no loop-carried state
    const int vb = blockIdx.x;
    TS(0);
    gemm256_tile<XR, WR, CONV, ACT, ROWB, LNF, EK>(p, vb, tiles_m, tiles_n, smem, false, -1, wave);
    TS(7);
  } else {
    // the fixed-kind epilogues chain the next tile's prologue (gemm256_tile); the generic (EK 0) one
    // does not (chaining the staged row store measured 4 % slower on proj, 106.0 -> 110.3 us, round 3)
    const bool chain = EK != 0;
    // dynamic schedule (vda_epilogue.sched; not with EK 3, whose row-bias slots follow the static tile
    // order): a block's first tile is its id, the rest of its XCD's tiles (grid + xcd + 8 v) go by ticket
    const bool dyn = XR == 2 && EK != 3 && p.epi.sched != nullptr && ntiles > (int)gridDim.x &&
                     (gridDim.x & 7) == 0;
    unsigned* tctr = dyn ? reinterpret_cast<unsigned*>(p.epi.sched) + (blockIdx.x & 7) : nullptr;
    const int tbase = (int)gridDim.x + (int)(blockIdx.x & 7);
    int* tslot = XR == 2 ? reinterpret_cast<int*>(smem + SMEM_HALVES - 64) : nullptr;
    bool pre = false;
    TSC(0);
    for (int vb = blockIdx.x; vb >= 0 && vb < ntiles;) {
      TS(0);
      const int nxt = vb + (int)gridDim.x;
      vb = gemm256_tile<XR, WR, CONV, ACT, ROWB, LNF, EK>(p, vb, tiles_m, tiles_n, smem, pre, nxt < ntiles ? nxt : -1,
                                                         wave, tctr, tbase, tslot);
      if (!chain) __syncthreads();
      pre = chain;
      TS(7);
    }
    TSC(1);
    if (dyn && wave == 0 && threadIdx.x == 0) {
      // the block has drawn its last ticket (retired by its tile's waits): the last block to leave zeroes
      // the counters for the next launch on this stream
      unsigned* sc = reinterpret_cast<unsigned*>(p.epi.sched);
      if (__hip_atomic_fetch_add(sc + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
#pragma unroll
        for (int i = 0; i < 9; ++i) __hip_atomic_store(sc + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// Knobs of the tuning build (include/vda_tune.h); compile-time constants in the product library.
VDA_KNOB(int, g_force_tile, -1);  // vda_debug_force_tile
VDA_KNOB(int, g_persist, -1);     // vda_debug_gemm_sched; -1 = automatic
VDA_KNOB(int, g_stagger, -1);
VDA_KNOB(int, g_desync, 0);       // vda_debug_gemm_desync
// vda_debug_gemm_epi: the residual + row-statistics GEMMs (proj / fc2) through the register epilogue
// (EK 2).  Off: bit-identical but measured slower than the staged epilogue (round 3: proj 94.8 -> 102.9
// us, fc2 320 -> 334 us; round 4 with whole-line stores / residual loads and asm LDS statistics: proj
// 104.9 -> 111.9, fc2 319.2 -> 331.2, same box, tools/ab_gemm.py, profiles/r04_ab_gemm_ek2.log): the
// residual loads issued at the epilogue start are waited for right away, where the staged epilogue
// covers them with its LDS staging pass.
VDA_KNOB(int, g_res_epi, 0);

int cu_count() { return vda_cu_count(); }

// grid and start stagger of a phased launch (see gemm256_kernel)
void phased_sched(int ntiles, int nk, bool conv, int& grid, int& ticks) {
  const int cus = cu_count();
  // measured in situ: persistent pays for the dense GEMMs, one block per tile for the convs
  const int persist = conv ? 0 : (g_persist >= 0 ? g_persist : cus);
  grid = persist == 0 ? ntiles : std::min(ntiles, persist);
  // The start stagger for a short last round (half the blocks with one tile fewer start half a
  // tile late, ~1.45 us per 64-deep K step + ~6 us prologue/epilogue) is off by default: it is worth
  // +0.4 % with one clip in flight but -0.6 % with the two clips in flight the drivers run (the
  // sleeping blocks hold CUs the other clip's kernels would use).  vda_debug_gemm_sched(-1, -2)
  // restores it, a value >= 0 forces that many 100-MHz ticks.
  ticks = 0;
  (void)nk;
  if (g_stagger >= 0) {
    ticks = g_stagger;
  } else if (g_stagger == -2 && ntiles > grid && ntiles % grid <= grid / 2) {
    ticks = (int)((nk * 1.45f + 6.f) * 0.5f * 100.f);
  }
}

template <int BM, int BN, int NWM, int NWN, int KB, int NS, bool CONV, int ACT>
void launch_tile(const GemmParams& p, hipStream_t st) {
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  hipLaunchKernelGGL((gemm_kernel<BM, BN, NWM, NWN, KB, NS, CONV, ACT>), dim3(tiles_m * tiles_n), dim3(NWM * NWN * 64),
                     0, st, p, tiles_m, tiles_n);
}

template <int XR, int WR, bool CONV, int ACT>
void launch_phased(const GemmParams& p, hipStream_t st) {
  const int BM = 128 * XR, BN = 128 * WR;
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  int grid, ticks;
  phased_sched(tiles_m * tiles_n, (p.K + 63) / 64, CONV, grid, ticks);
  if constexpr (!CONV && ACT == VDA_ACT_NONE && XR == 2) {
    if (p.epi.rowbias && p.epi.ln_stats) {  // LN fold + per-frame row bias (motion-module q/k/v), EK 3
      hipLaunchKernelGGL((gemm256_kernel<XR, WR, CONV, ACT, false, true, 3>), dim3(grid), dim3(512), 0, st, p, tiles_m,
                         tiles_n, ticks, g_desync);
      return;
    }
  }
  if constexpr (!CONV && ACT == VDA_ACT_NONE) {
    if (p.epi.rowbias) {
      hipLaunchKernelGGL((gemm256_kernel<XR, WR, CONV, ACT, true>), dim3(grid), dim3(512), 0, st, p, tiles_m, tiles_n, ticks,
                         g_desync);
      return;
    }
  }
  if constexpr (!CONV && XR == 2 && ACT == VDA_ACT_GEGLU) {
    if (p.epi.ln_stats) {  // LN fold + GEGLU (the motion modules' ff_norm -> ff.net[0]), staged epilogue
      hipLaunchKernelGGL((gemm256_kernel<XR, WR, CONV, ACT, false, true>), dim3(grid), dim3(512), 0, st, p, tiles_m, tiles_n,
                         ticks, g_desync);
      return;
    }
  }
  if constexpr (!CONV && XR == 2 && (ACT == VDA_ACT_NONE || ACT == VDA_ACT_GELU)) {
    const vda_epilogue& e = p.epi;
    const bool rows1 = e.store == VDA_STORE_ROWS && e.bias && !e.gamma && !e.res2 && !e.rowbias;
    if (e.ln_stats) {
      if (rows1 && !e.res && !e.stats_out)
        hipLaunchKernelGGL((gemm256_kernel<XR, WR, CONV, ACT, false, true, 1>), dim3(grid), dim3(512), 0, st, p, tiles_m,
                           tiles_n, ticks, g_desync);
      else
        hipLaunchKernelGGL((gemm256_kernel<XR, WR, CONV, ACT, false, true>), dim3(grid), dim3(512), 0, st, p, tiles_m, tiles_n,
                           ticks, g_desync);
      return;
    }
    if (rows1 && !e.res && !e.stats_out) {
      hipLaunchKernelGGL((gemm256_kernel<XR, WR, CONV, ACT, false, false, 1>), dim3(grid), dim3(512), 0, st, p, tiles_m,
                         tiles_n, ticks, g_desync);
      return;
    }
    if constexpr (ACT == VDA_ACT_NONE) {
      if (g_res_epi && rows1 && e.res && e.stats_out) {
        hipLaunchKernelGGL((gemm256_kernel<XR, WR, CONV, ACT, false, false, 2>), dim3(grid), dim3(512), 0, st, p, tiles_m,
                           tiles_n, ticks, g_desync);
        return;
      }
    }
  }
  hipLaunchKernelGGL((gemm256_kernel<XR, WR, CONV, ACT, false>), dim3(grid), dim3(512), 0, st, p, tiles_m, tiles_n, ticks,
                     g_desync);
}

template <bool CONV, int ACT>
int launch_act(const GemmParams& p, hipStream_t st) {  // returns the tile configuration it launched
  int cfg = g_force_tile;
  if (cfg < 0) {
    // measured on MI355X (tools/archive/bench_gemm.py): 256x256 wins every large-N shape; N = 128 prefers
    // 256x128; short K (<= 256) and narrow N prefer the 2-blocks-per-CU 128x64 tile.
    const vda_epilogue& e = p.epi;
    const bool a16 = ((uintptr_t)p.y % 16 == 0) && p.ldy % 8 == 0 && p.N % 8 == 0 &&
                     (!e.res || ((uintptr_t)e.res % 16 == 0 && e.ldres % 8 == 0)) &&
                     (!e.res2 || ((uintptr_t)e.res2 % 16 == 0 && e.ldres2 % 8 == 0)) &&
                     (e.act != VDA_ACT_GEGLU || (p.N / 2) % 8 == 0);
    // the phased kernels' dense path needs K % 64 == 0 and 32-bit buffer offsets
    // (per-row bias only in the dense, activation-free phased instantiation)
    const bool dense_ok = (CONV || (p.K % 64 == 0 && (long)p.M * p.ldx * 2 < (1L << 31) &&
                                    (long)p.N * p.K * 2 < (1L << 31))) &&
                          (!e.rowbias || (!CONV && ACT == VDA_ACT_NONE));
    if (p.N <= 64 || (p.K <= 256 && p.N < 256)) cfg = 2;
    else if (p.N >= 256 && p.M >= 4096 && dense_ok && (e.store != VDA_STORE_ROWS || a16)) cfg = 4;
    else if (p.N == 128 && p.M >= 8192 && a16 && dense_ok && e.store == VDA_STORE_ROWS && !e.ln_stats) cfg = 5;
    else if (p.N >= 256 && p.M >= 4096) cfg = 3;
    else if (p.N >= 128 && p.M >= 4096) cfg = 1;
    else if (CONV) cfg = 0;
    else {
      // small M (the streaming mode's one-frame encoder, M = 1,370): the largest tile that still
      // gives >= 2 tiles per CU, else 64x64 (tools/archive/bench_gemm_small.py: ViT-L fc2 72.8 -> 43.5 us,
      // proj 24.0 -> 14.0, qkv 29.5 -> 25.0, fc1 34.2 -> 30.3)
      const long ncu2 = 2L * cu_count();
      auto ntiles = [&](int bm, int bn) { return (long)((p.M + bm - 1) / bm) * ((p.N + bn - 1) / bn); };
      cfg = ntiles(128, 128) >= ncu2 ? 0 : ntiles(128, 64) >= ncu2 ? 2 : 6;
    }
  }
  switch (cfg) {
    case 1: launch_tile<256, 128, 4, 2, 32, 4, CONV, ACT>(p, st); break;
    case 2: launch_tile<128, 64, 2, 2, 32, 4, CONV, ACT>(p, st); break;
    case 3: launch_tile<256, 256, 2, 4, 32, 4, CONV, ACT>(p, st); break;
    case 4: launch_phased<2, 2, CONV, ACT>(p, st); break;
    case 5: launch_phased<4, 1, CONV, ACT>(p, st); break;
    case 6: launch_tile<64, 64, 2, 2, 32, 4, CONV, ACT>(p, st); break;
    case 7: launch_tile<64, 128, 2, 2, 32, 4, CONV, ACT>(p, st); break;
    default: launch_tile<128, 128, 2, 2, 32, 4, CONV, ACT>(p, st); break;
  }
  return cfg;
}

template <bool CONV>
int launch(const GemmParams& p, hipStream_t st) {
  int cfg;
  switch (p.epi.act) {
    case VDA_ACT_GELU: cfg = launch_act<CONV, VDA_ACT_GELU>(p, st); break;
    case VDA_ACT_GEGLU: cfg = launch_act<CONV, VDA_ACT_GEGLU>(p, st); break;
    case VDA_ACT_RELU: cfg = launch_act<CONV, VDA_ACT_RELU>(p, st); break;
    default: cfg = launch_act<CONV, VDA_ACT_NONE>(p, st); break;
  }
  VDA_LAUNCH_CHECK();
  if (p.epi.stats_out) {
    // the phased 256x256 dense activation-free kernel with at most one residual writes the partial
    // row statistics in its epilogue; any other route gets them from a separate partial-sum pass
    const int nres = (p.epi.res ? 1 : 0) + (p.epi.res2 ? 1 : 0);
    const bool in_epi = !CONV && cfg == 4 && p.epi.act == VDA_ACT_NONE && !p.epi.rowbias && !p.epi.ln_stats && nres <= 1;
    if (!in_epi) return vda_row_partials_launch(p.y, p.ldy, p.epi.stats_out, p.M, p.N, st);
  }
  return 0;
}

int launch_reg_conv(const GemmParams& p, hipStream_t st) {
  const int tiles_m = (p.M + 127) / 128;
  if (p.N >= 128) {
    const int tiles_n = (p.N + 127) / 128;
    if (p.epi.act == VDA_ACT_RELU)
      hipLaunchKernelGGL((gemm_reg_kernel<128, 128, ConvLoader, VDA_ACT_RELU>), dim3(tiles_m * tiles_n), dim3(256), 0, st, p, tiles_n);
    else
      hipLaunchKernelGGL((gemm_reg_kernel<128, 128, ConvLoader, VDA_ACT_NONE>), dim3(tiles_m * tiles_n), dim3(256), 0, st, p, tiles_n);
  } else {
    const int tiles_n = (p.N + 63) / 64;
    if (p.epi.act == VDA_ACT_RELU)
      hipLaunchKernelGGL((gemm_reg_kernel<128, 64, ConvLoader, VDA_ACT_RELU>), dim3(tiles_m * tiles_n), dim3(256), 0, st, p, tiles_n);
    else
      hipLaunchKernelGGL((gemm_reg_kernel<128, 64, ConvLoader, VDA_ACT_NONE>), dim3(tiles_m * tiles_n), dim3(256), 0, st, p, tiles_n);
  }
  VDA_LAUNCH_CHECK();
  return 0;
}

vda_epilogue default_epi() {
  vda_epilogue e{};
  e.rdiv = 1; e.rmod = 1;
  return e;
}

int check_epi(const vda_epilogue& e, int M, int N) {
  VDA_CHECK_ARG(!e.rowbias || (e.rdiv > 0 && e.rmod > 0), "rowbias needs rdiv, rmod > 0");
  VDA_CHECK_ARG(e.act >= 0 && e.act <= 3, "unknown activation");
  VDA_CHECK_ARG(e.act != VDA_ACT_GEGLU || (N % 32 == 0 && !e.rowbias && e.store == 0 && !e.res2),
                "GEGLU needs N % 32 == 0, no rowbias/res2, row store");
  VDA_CHECK_ARG(e.store == VDA_STORE_ROWS ||
                (e.store == VDA_STORE_PIXEL_SHUFFLE && e.ps_k > 0 && e.ps_cout > 0 && e.ps_cout % 4 == 0 &&
                 e.ps_hin > 0 && e.ps_win > 0 && N == e.ps_k * e.ps_k * e.ps_cout && !e.res && !e.res2),
                "bad pixel-shuffle store geometry");
  // the LN fold exists for the activation-free, GELU and GEGLU epilogues (every kernel route applies it
  // there; anything else would silently run an un-normalised GEMM); with a row bias only on the
  // phased route's EK 3 epilogue (vda_gemm checks the shape)
  VDA_CHECK_ARG(!e.ln_stats || (e.ln_colsum && e.store == VDA_STORE_ROWS && !e.gamma &&
                                 (e.act == VDA_ACT_NONE || e.act == VDA_ACT_GELU || e.act == VDA_ACT_GEGLU)),
                "ln_stats needs ln_colsum, a row store, no gamma, activation none / gelu / geglu");
  VDA_CHECK_ARG(!e.ln_stats || !e.rowbias ||
                    (e.act == VDA_ACT_NONE && e.bias && !e.res && !e.res2 && !e.stats_out && e.rdiv >= 256),
                "ln_stats with rowbias needs a bias, no activation / residual / stats_out, rdiv >= 256");
  VDA_CHECK_ARG(!e.ln_stats || (e.ln_parts >= 0 && e.ln_parts <= 4), "ln_parts must be 0 .. 4");
  // the phased route stages the statistics in 16-byte pieces, reading the last one 8 B early when the
  // float count is not a multiple of 4: the buffer must hold at least one whole piece (M * P >= 2)
  VDA_CHECK_ARG(!e.ln_stats || (long)M * (e.ln_parts > 0 ? e.ln_parts : 1) >= 2, "ln_stats needs M * max(ln_parts, 1) >= 2");
  VDA_CHECK_ARG(!e.stats_out || (e.store == VDA_STORE_ROWS && e.act != VDA_ACT_GEGLU),
                "stats_out needs a row store and no GEGLU");
  VDA_CHECK_ARG(!e.res || e.ldres % 4 == 0, "ldres % 4");
  VDA_CHECK_ARG(!e.res2 || e.ldres2 % 4 == 0, "ldres2 % 4");
  return 0;
}

}  // namespace

extern "C" int vda_gemm(const void* x, int64_t ldx, const void* w, void* y, int64_t ldy, int32_t M,
                        int32_t N, int32_t K, const vda_epilogue* epi, void* stream) {
  VDA_CHECK_ARG(x && w && y, "null pointer");
  VDA_CHECK_ARG(M > 0 && N > 0 && K > 0, "empty GEMM");
  VDA_CHECK_ARG(K % 8 == 0 && ldx % 8 == 0 && ldx >= K, "K and ldx must be multiples of 8, ldx >= K");
  VDA_CHECK_ARG(N % 4 == 0 && ldy % 4 == 0, "N and ldy must be multiples of 4");
  GemmParams p{};
  p.x = (const h16*)x; p.ldx = ldx; p.w = (const h16*)w; p.y = (h16*)y; p.ldy = ldy;
  p.M = M; p.N = N; p.K = K;
  p.epi = epi ? *epi : default_epi();
  if (p.epi.rdiv <= 0) p.epi.rdiv = 1;
  if (p.epi.rmod <= 0) p.epi.rmod = 1;
  VDA_CHECK_ARG(p.epi.res2_h == 0 && p.epi.res2_w == 0, "upsampled res2: vda_conv2d only");
  if (p.epi.drop_period != 0) {  // only the phased route's register LN-fold epilogue (EK 1) drops rows
    const vda_epilogue& e = p.epi;
    VDA_CHECK_ARG(e.drop_period >= 256 && e.ln_stats && e.ln_colsum && e.bias && e.act == VDA_ACT_NONE &&
                      e.store == VDA_STORE_ROWS && !e.gamma && !e.res && !e.res2 && !e.rowbias && !e.stats_out &&
                      N % 256 == 0 && M >= 4096 && K % 64 == 0 && (long)M * ldx * 2 < (1L << 31) &&
                      (long)N * K * 2 < (1L << 31) && (uintptr_t)y % 16 == 0 && ldy % 8 == 0 && g_force_tile < 0,
                  "drop_period: >= 256, with ln_stats + bias, no activation / gamma / res / rowbias / stats_out, "
                  "N % 256 == 0, M >= 4096, K % 64 == 0, 16-byte aligned rows");
  }
  int rc = check_epi(p.epi, M, N);
  if (rc) return rc;
  if (p.epi.ln_stats && p.epi.rowbias) {  // only the phased 256x256 route (EK 3) implements the pair
    const bool a16 = ((uintptr_t)p.y % 16 == 0) && ldy % 8 == 0 && ((uintptr_t)p.x % 16 == 0);
    VDA_CHECK_ARG(N % 256 == 0 && M >= 4096 && K % 64 == 0 && a16 && (long)M * ldx * 2 < (1L << 31) &&
                      (long)N * K * 2 < (1L << 31) && g_force_tile == -1,
                  "ln_stats with rowbias needs N % 256 == 0, M >= 4096, K % 64 == 0, 16-B aligned rows");
  }
  return launch<false>(p, (hipStream_t)stream);
}

// The strip-tiled 3x3 conv (vda_strip.hip) serves 3x3 / s1 / p1 convs with 256 output channels and
// Cin >= 512 on maps up to 160 wide (layer2..4_rn; measured 10-14% faster there, 1-4% slower than the
// implicit GEMM at Cin = 256), and any Cout = 256 3x3 conv whose 256-pixel strip tiles would fill at
// most half the CUs (19^2 maps: the strip kernel then splits the input channels over several work
// items).  vda_debug_force_tile(-3) routes every Cout = 256 conv to it, (-2) none.
static bool conv_takes_strip(int BT, int H, int W, int Cin, int Cout, int ks, int stride, int pad, int up_h) {
  if (up_h > 0 || ks != 3 || stride != 1 || pad != 1 || !vda_conv_strip_serves(W, Cin, Cout)) return false;
  const long strip_tiles = (long)BT * ((H * W + 255) / 256);
  return g_force_tile == -3 || (g_force_tile == -1 && (Cin >= 512 || strip_tiles * 2 <= cu_count()));
}

// Stride-2 3x3 convs (the DPT reassemble's resize_layers[3], dpt.py:77-82: 1024 -> 1024 at 37^2 -> 19^2):
// explicit im2col into the workspace + the dense phased GEMM.  The implicit-GEMM conv runs its K steps at
// about half the dense rate, and at 184 tiles x 144 K steps (32 frames) the copy costs far less than that
// (410 -> 210 us of GEMM for ~70 us of copy, tools/archive/s2conv_probe.py); bit-identical (same K order).
static long conv_im2col_bytes(int BT, int H, int W, int Cin, int ks, int stride, int pad) {
  const long Ho = (H + 2L * pad - ks) / stride + 1, Wo = (W + 2L * pad - ks) / stride + 1;
  return (long)BT * Ho * Wo * ks * ks * Cin * 2;
}
static bool conv_takes_im2col(int BT, int H, int W, int Cin, int Cout, int ks, int stride, int pad, int up_h) {
  if (up_h > 0 || ks != 3 || stride != 2 || Cin % 64 != 0 || Cout % 256 != 0 || g_force_tile != -1) return false;
  const long Ho = (H + 2L * pad - ks) / stride + 1, Wo = (W + 2L * pad - ks) / stride + 1;
  const long M = (long)BT * Ho * Wo;
  return Ho > 0 && Wo > 0 && M >= 4096 && conv_im2col_bytes(BT, H, W, Cin, ks, stride, pad) < (1L << 31);
}

// the halo-tiled 256-channel conv route (the only one whose epilogue reads an upsampled res2)
static bool conv_takes_hconv(int BT, int H, int W, int Cin, int Cout, int ks, int stride, int pad) {
  return ks == 3 && stride == 1 && pad == 1 && g_force_tile == -1 && vda_conv_hconv_serves(BT, H, W, Cin, Cout);
}

extern "C" int64_t vda_conv2d_workspace(int32_t BT, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t ks,
                                        int32_t stride, int32_t pad) {
  if (BT <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0) return 0;
  if (conv_takes_hconv(BT, H, W, Cin, Cout, ks, stride, pad)) return 0;
  if (conv_takes_im2col(BT, H, W, Cin, Cout, ks, stride, pad, 0)) return conv_im2col_bytes(BT, H, W, Cin, ks, stride, pad);
  if (!conv_takes_strip(BT, H, W, Cin, Cout, ks, stride, pad, 0)) return 0;
  return vda_conv_strip_ws_bytes(BT, H, W, Cin, Cout);
}

extern "C" int vda_conv2d_res2_upsample_ok(int32_t BT, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t ks,
                                           int32_t stride, int32_t pad) {
  if (BT <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0) return 0;
  return conv_takes_hconv(BT, H, W, Cin, Cout, ks, stride, pad) ? 1 : 0;
}

extern "C" int vda_conv2d(const void* x, const void* w, void* y, int32_t BT, int32_t H, int32_t W,
                          int32_t Cin, int32_t Cout, int32_t ks, int32_t stride, int32_t pad,
                          int32_t pre_relu, int32_t up_h, int32_t up_w, const vda_epilogue* epi,
                          void* ws, int64_t ws_bytes, void* stream) {
  VDA_CHECK_ARG(x && w && y, "null pointer");
  VDA_CHECK_ARG(BT > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && ks > 0 && stride > 0 && pad >= 0,
                "bad conv geometry");
  VDA_CHECK_ARG(Cin % 8 == 0 && Cout % 4 == 0, "Cin % 8 and Cout % 4 required");
  const int Hi = up_h > 0 ? up_h : H, Wi = up_w > 0 ? up_w : W;
  GemmParams p{};
  p.x = (const h16*)x; p.w = (const h16*)w; p.y = (h16*)y;
  p.H = H; p.W = W; p.Cin = Cin; p.ks = ks; p.stride = stride; p.pad = pad; p.pre_relu = pre_relu;
  p.up_h = up_h > 0 ? up_h : 0; p.up_w = up_w > 0 ? up_w : 0;
  p.Ho = (Hi + 2 * pad - ks) / stride + 1;
  p.Wo = (Wi + 2 * pad - ks) / stride + 1;
  VDA_CHECK_ARG(p.Ho > 0 && p.Wo > 0, "empty conv output");
  p.M = BT * p.Ho * p.Wo; p.N = Cout; p.K = ks * ks * Cin;
  p.ldy = Cout; p.ldx = 0;
  p.epi = epi ? *epi : default_epi();
  if (p.epi.rdiv <= 0) p.epi.rdiv = 1;
  if (p.epi.rmod <= 0) p.epi.rmod = 1;
  VDA_CHECK_ARG(p.epi.store == VDA_STORE_ROWS && (p.epi.act == VDA_ACT_NONE || p.epi.act == VDA_ACT_RELU),
                "conv: row store, activation none/relu");
  VDA_CHECK_ARG(!p.epi.stats_out && !p.epi.ln_stats, "conv: no LayerNorm fold / row statistics");
  int rc = check_epi(p.epi, p.M, Cout);
  if (rc) return rc;
  const bool res2_up = p.epi.res2_h > 0 || p.epi.res2_w > 0;
  if (res2_up) {  // refinenet1's skip add on the previous block's output, upsampled in the epilogue
    VDA_CHECK_ARG(p.epi.res2 && p.epi.res2_h > 0 && p.epi.res2_w > 0 && p.epi.ldres2 == Cout && p.up_h == 0 &&
                      !p.epi.gamma && !p.epi.rowbias && (!p.epi.res || p.epi.ldres == Cout) &&
                      p.epi.res2_h <= p.Ho && p.epi.res2_w <= p.Wo &&
                      (long)p.epi.res2_h * p.epi.res2_w * Cout * 2 < (1L << 31) &&
                      conv_takes_hconv(BT, H, W, Cin, Cout, ks, stride, pad),
                  "upsampled res2 needs the halo conv route (vda_conv2d_res2_upsample_ok), a [BT, h <= Ho, w <= Wo, "
                  "Cout] source, no gamma / rowbias / input upsample");
    return vda_conv_hconv(x, w, y, p.epi.bias, p.epi.act == VDA_ACT_RELU, pre_relu, p.epi.res, p.epi.res2,
                          p.epi.res2_h, p.epi.res2_w, BT, H, W, Cin, Cout, (hipStream_t)stream);
  }
  if (p.up_h > 0) {
    // 3x3 conv on a bilinear resize with 128 outputs (output_conv1 on refinenet1's x2 resize): the
    // halo conv with the resize fused into its patch staging (bit-identical to resize + conv)
    if (g_force_tile < 0 && ks == 3 && stride == 1 && pad == 1 && !pre_relu && !p.epi.res && !p.epi.res2 &&
        !p.epi.gamma && !p.epi.rowbias) {
      rc = vda_conv_halo_fused(x, w, y, p.epi.bias, p.epi.act == VDA_ACT_RELU, BT, H, W, p.up_h, p.up_w, Cin, Cout,
                               (hipStream_t)stream);
      if (rc != 1) return rc;
    }
    return launch_reg_conv(p, (hipStream_t)stream);
  }
  // large maps with 256 output channels (the refinenet RCU convs and layer1_rn at 148^2): the
  // halo-tiled phased conv stages each input patch once per 64-channel slab instead of 9 times
  if (!p.epi.gamma && !p.epi.rowbias && (!p.epi.res || p.epi.ldres == Cout) && (!p.epi.res2 || p.epi.ldres2 == Cout) &&
      conv_takes_hconv(BT, H, W, Cin, Cout, ks, stride, pad)) {
    rc = vda_conv_hconv(x, w, y, p.epi.bias, p.epi.act == VDA_ACT_RELU, pre_relu, p.epi.res, p.epi.res2, 0, 0, BT, H,
                        W, Cin, Cout, (hipStream_t)stream);
    if (rc != 1) return rc;
  }
  if (conv_takes_strip(BT, H, W, Cin, Cout, ks, stride, pad, 0) && !p.epi.gamma && !p.epi.rowbias &&
      (!p.epi.res || p.epi.ldres == Cout) && (!p.epi.res2 || p.epi.ldres2 == Cout)) {
    rc = vda_conv_strip(x, w, y, p.epi.bias, p.epi.act == VDA_ACT_RELU, pre_relu, p.epi.res, p.epi.res2, BT, H, W,
                        Cin, Cout, ws, ws ? ws_bytes : 0, (hipStream_t)stream);
    if (rc != 1) return rc;
  }
  // large 3x3 maps with 128 output channels (output_conv1 at 296^2): halo-tiled kernel (vda_depth.hip)
  if (g_force_tile < 0 && ks == 3 && stride == 1 && pad == 1 && !pre_relu && !p.epi.res && !p.epi.res2 &&
      !p.epi.gamma && !p.epi.rowbias && (long)H * W >= 128L * 128L) {
    rc = vda_conv_halo(x, w, y, p.epi.bias, p.epi.act == VDA_ACT_RELU, BT, H, W, Cin, Cout, (hipStream_t)stream);
    if (rc != 1) return rc;
  }
  if (conv_takes_im2col(BT, H, W, Cin, Cout, ks, stride, pad, 0) && !pre_relu && ws &&
      ws_bytes >= conv_im2col_bytes(BT, H, W, Cin, ks, stride, pad) && (uintptr_t)ws % 16 == 0 &&
      (uintptr_t)x % 16 == 0) {
    rc = vda_conv_im2col(x, ws, BT, H, W, Cin, p.Ho, p.Wo, ks, stride, pad, (hipStream_t)stream);
    if (rc) return rc;
    p.x = (const h16*)ws;
    p.ldx = p.K;
    return launch<false>(p, (hipStream_t)stream);
  }
  return launch<true>(p, (hipStream_t)stream);
}


extern "C" int vda_depth_head(const void* x, const void* w1, const float* b1, const float* w2, const float* b2,
                              float* depth, void* ws, int32_t BT, int32_t Hin, int32_t Win, int32_t C, int32_t Ho,
                              int32_t Wo, void* stream) {
  VDA_CHECK_ARG(x && w1 && b1 && w2 && b2 && depth, "null pointer");
  VDA_CHECK_ARG(BT > 0 && Hin > 0 && Win > 0 && Ho > 0 && Wo > 0, "bad depth-head geometry");
  VDA_CHECK_ARG(C % 8 == 0, "depth head needs C % 8 == 0");
  hipStream_t st = (hipStream_t)stream;
  int rc;
  // default: the depth conv of vda_dconv.hip (two 4-wave blocks per CU, 64 pixels x all 64 hi/lo rows
  // per wave) with the bilinear resize fused into its patch building (the resized map is never
  // written); vda_debug_dconv(2): bilinear resize into ws + the same conv on the materialised map
  // (bit-identical); vda_debug_dconv(0): the older 8-wave halo kernels below.
  if (g_force_tile == -1) {
    rc = vda_depth_conv_fused(x, w1, b1, w2, b2, depth, BT, Hin, Win, Ho, Wo, C, st);
    if (rc != 1) return rc;
  }
  if (g_force_tile == -1 && vda_depth_conv_serves(Ho, Wo, C)) {
    VDA_CHECK_ARG(ws, "depth head: needs the resize workspace (vda_depth_head_workspace)");
    rc = vda_upsample_bilinear(x, ws, BT, Hin, Win, C, Ho, Wo, stream);
    if (rc) return rc;
    rc = vda_depth_conv(ws, w1, b1, w2, b2, depth, BT, Ho, Wo, C, st);
    if (rc != 1) return rc;
  }
  // 0) resize fused into the halo conv's patch staging (the resized map is never written;
  //    bit-identical to 1 + 2).  vda_debug_force_tile(9) takes the materialised path below.
  if (g_force_tile < 9) {
    rc = vda_depth_halo_fused(x, w1, b1, w2, b2, depth, BT, Hin, Win, Ho, Wo, C, st);
    if (rc != 1) return rc;
  }
  VDA_CHECK_ARG(ws, "depth head: this shape needs the resize workspace (vda_depth_head_workspace)");
  // 1) bilinear (align_corners=True) resize of the output_conv1 map to (Ho, Wo), fp16 like the
  //    reference's autocast interpolate (dpt_temporal.py:92-94)
  rc = vda_upsample_bilinear(x, ws, BT, Hin, Win, C, Ho, Wo, stream);
  if (rc) return rc;
  // 2) 3x3 conv C -> 32 with split-fp16 weights + fused ReLU / 1x1 / ReLU epilogue: the halo-tiled
  //    kernel (vda_depth.hip) unless a tuning override asks for the implicit-GEMM one
  if (g_force_tile < 10) {
    rc = vda_depth_halo(ws, w1, b1, w2, b2, depth, BT, Ho, Wo, C, st);
    if (rc != 1) return rc;
  }
  GemmParams p{};
  p.x = (const h16*)ws; p.w = (const h16*)w1; p.y = (h16*)depth;
  p.H = Ho; p.W = Wo; p.Cin = C; p.ks = 3; p.stride = 1; p.pad = 1; p.pre_relu = 0;
  p.Ho = Ho; p.Wo = Wo;
  p.M = BT * Ho * Wo; p.N = 64; p.K = 9 * C; p.ldy = 1;
  p.epi = default_epi();
  p.epi.bias = b1; p.epi.gamma = w2; p.epi.rowbias = b2;
  const int cfg = g_force_tile >= 10 ? g_force_tile - 10 : 3;
  switch (cfg) {
    case 1: {
      const int tiles_m = (p.M + 255) / 256;
      hipLaunchKernelGGL((gemm_kernel<256, 64, 8, 1, 64, 3, true, ACT_DEPTH>), dim3(tiles_m), dim3(512), 0, st, p, tiles_m, 1);
      break;
    }
    case 2: {
      const int tiles_m = (p.M + 511) / 512;
      hipLaunchKernelGGL((gemm_kernel<512, 64, 8, 1, 64, 2, true, ACT_DEPTH>), dim3(tiles_m), dim3(512), 0, st, p, tiles_m, 1);
      break;
    }
    case 3: {
      const int tiles_m = (p.M + 255) / 256;
      hipLaunchKernelGGL((gemm_kernel<256, 64, 8, 1, 64, 2, true, ACT_DEPTH>), dim3(tiles_m), dim3(512), 0, st, p, tiles_m, 1);
      break;
    }
    default: {
      const int tiles_m = (p.M + 127) / 128;
      hipLaunchKernelGGL((gemm_kernel<128, 64, 4, 1, 32, 4, true, ACT_DEPTH>), dim3(tiles_m), dim3(256), 0, st, p, tiles_m, 1);
    }
  }
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int64_t vda_depth_head_workspace(int32_t BT, int32_t Hin, int32_t Win, int32_t C, int32_t Ho, int32_t Wo) {
  if (BT <= 0 || Hin <= 0 || Win <= 0 || C <= 0 || Ho <= 0 || Wo <= 0) return 0;
  if (g_force_tile == -1 && vda_depth_conv_fused_serves(Hin, Win, Ho, Wo, C)) return 0;  // fused: no resized map
  if (g_force_tile == -1 && vda_depth_conv_serves(Ho, Wo, C)) return (int64_t)BT * Ho * Wo * C * 2;
  if (g_force_tile < 9 && vda_depth_halo_fused_serves(Hin, Win, Ho, Wo, C)) return 0;  // fused: no resized map
  return (int64_t)BT * Ho * Wo * C * 2;
}

#ifdef VDA_TUNING
extern "C" int vda_debug_force_tile(int32_t cfg) {
  g_force_tile = cfg;
  return 0;
}

extern "C" int vda_debug_gemm_desync(int32_t groups) {
  g_desync = groups;
  return 0;
}

extern "C" int vda_debug_gemm_sched(int32_t persist_blocks, int32_t stagger) {
  g_persist = persist_blocks;
  g_stagger = stagger;
  return 0;
}

extern "C" int vda_debug_gemm_epi(int32_t res_register) {
  g_res_epi = res_register;
  return 0;
}
#endif
