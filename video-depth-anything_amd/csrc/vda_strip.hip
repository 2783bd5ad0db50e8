// 3x3 / stride 1 / pad 1 convolutions with 256 output channels on maps up to 160 pixels wide (the
// DPT head's layerN_rn convs and FeatureFusionBlock ResidualConvUnits at 148^2 / 74^2 / 37^2 / 19^2,
// blocks.py:20-32, :68-91) as a halo-staged "strip" conv.
//
// A tile is 256 consecutive output pixels of one frame in row-major order (so no tile edge is wasted
// on maps whose width is not a multiple of 16, e.g. 148 = 9.25 x 16).  Those pixels span at most
// 3 image rows; the rows above and below plus one halo column each side (<= 5 x (W+2) pixels) are
// staged ONCE per 32-channel slab by LDS-DMA and all 9 taps read them from LDS: input traffic ~2x the
// map instead of the implicit GEMM's 9x.  Weights stream per (slab, tap) step (256 rows x 32 channels
// = 16 KB) from L2.  Block = 8 waves, persistent; wave w: 4 m-blocks (64 pixels, mg = w & 3) x 8
// n-blocks (128 channels, ng = w >> 2), 16x16x32 fp16 MFMA with W as the A operand (a lane owns 4
// consecutive channels of one pixel).  Per step each wave issues 2 weight pieces and, on a slab's
// first step, 7 pieces of the next slab's patch (fixed count: pieces past the patch reload the zero
// page into spare slots), so every vmcnt is a constant; one raw s_barrier per step.
// Epilogue: +bias, [ReLU], fp16 round, then + res + res2 as fp16 adds (the reference's fp16
// residual adds, as in the GEMM epilogue); pre-ReLU (RCU, blocks.py:78) is applied to the X
// fragments as they are read.
//
// Split over channel slabs: a small map has too few tiles for the chip (19^2 x 32 frames = 64 tiles
// on 256 CUs: layer4_rn ran 310 us for 54 GFLOP).  A work item is then (tile, split): split s sums
// slabs [s*nsl, (s+1)*nsl) and stores its fp32 partial tile into its own workspace slice with plain
// stores; strip_finish_kernel adds the slices in a fixed order (deterministic) and applies the
// epilogue.  The host picks the split count from a rounds x steps cost model (vda_conv_strip).
#include "vda_common.h"
#include "../../include/vda.h"

namespace {

__device__ __attribute__((aligned(64))) uint4 g_sz_page[4];

constexpr int ST_M = 256;               // output pixels per tile
constexpr int ST_SLAB = 32;             // channels per staged slab
constexpr int ST_CPX = ST_SLAB / 8;     // 16-B chunks per pixel per slab (4)
constexpr int ST_MAXW = 160;            // widest map served
constexpr int ST_MAXPIX = 5 * (ST_MAXW + 2);                // patch pixels (<= 5 rows of W+2)
constexpr int ST_PP = (ST_MAXPIX * ST_CPX + 63) / 64;       // 1-KiB pieces per patch slab (51)
constexpr int ST_PPW = (ST_PP + 7) / 8;                     // per wave, fixed (7)
constexpr int ST_PBUF = ST_PPW * 8 * 512;                   // halfs per patch ring slot (56 KiB)
constexpr int ST_N = 256;                                   // output channels
constexpr int ST_WBUF = ST_N * ST_CPX * 8;                  // halfs per weight step (16 KiB)
constexpr int ST_WR = 3;                                    // weight ring: step t+2's weights in flight

struct StripParams {
  const h16* x;
  const h16* w;  // [256, 3, 3, Cin]
  h16* y;
  const float* bias;
  const h16* res;
  const h16* res2;
  float* ws;     // split > 1: [nsplit][BT * H * W][256] fp32 partial sums
  long ws_slice; // BT * H * W * 256
  int H, W, Cin;
  int pre_relu, relu_out;
  int tiles_per_frame, ntiles;
  int nsplit, nsl;  // channel-slab splits per tile, slabs per split
};

__device__ __forceinline__ void st_glds16(const void* src, h16* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (VDA_LDS void*)lds_base, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void st_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ int st_ppos(int pp, int cd) { return cd ^ ((pp >> 1) & 3); }
__device__ __forceinline__ int st_wpos(int n, int cd) { return cd ^ ((n >> 1) & 3); }

__global__ __launch_bounds__(512) void strip_conv_kernel(StripParams p) {
  __shared__ __attribute__((aligned(16))) h16 sm[2 * ST_PBUF + ST_WR * ST_WBUF];  // 160 KiB with 3 slots
  h16* patch = sm;
  h16* wbuf = sm + 2 * ST_PBUF;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mg = wave & 3, ng = wave >> 2;
  const int W = p.W, H = p.H, HW = p.H * p.W, PW = p.W + 2;
  const int nsl = p.nsl;                 // slabs per work item (all Cin / 32 when unsplit)
  const int K = 9 * p.Cin;
  const int nitems = p.ntiles * p.nsplit;
  const int my_items = (int)blockIdx.x < nitems ? (nitems - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int my_units = my_items * nsl;
  if (my_units == 0) return;
  const int my_steps = my_units * 9;
  const void* zero = (const void*)g_sz_page;

  // unit u of this block -> work item (tile, split) -> frame bt, first pixel q0, split index
  auto item_of_unit = [&](int u, int& bt, int& q0, int& sp) {
    const int it = (int)blockIdx.x + (u / nsl) * (int)gridDim.x;
    const int t = it / p.nsplit;
    sp = it - t * p.nsplit;
    bt = t / p.tiles_per_frame;
    q0 = (t - bt * p.tiles_per_frame) * ST_M;
  };
  auto slab_of_unit = [&](int u) {
    const int it = (int)blockIdx.x + (u / nsl) * (int)gridDim.x;
    return (it % p.nsplit) * nsl + u % nsl;
  };
  // patch of unit u -> ring slot (u & 1): image rows r0-1 .. r0-1+nrows-1, columns -1 .. W
  auto dma_patch = [&](int u, int j) {
    int bt, q0, sp;
    item_of_unit(u, bt, q0, sp);
    const int slab = sp * nsl + u % nsl;
    const int r0 = q0 / W;
    const int q1 = min(q0 + ST_M, HW) - 1;
    const int npix = (q1 / W - r0 + 3) * PW;
    const int q = wave + j * 8;  // piece index (fixed count per wave; pieces past the patch load zeros)
    const int s = q * 64 + lane;
    const int pp = s / ST_CPX, pos = s - pp * ST_CPX;
    const int cd = st_ppos(pp, pos);
    const int prow = pp / PW;
    const int iy = r0 - 1 + prow, ix = pp - prow * PW - 1;
    const void* src = zero;
    if (pp < npix && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
      src = p.x + (((long)bt * H + iy) * W + ix) * p.Cin + slab * ST_SLAB + cd * 8;
    st_glds16(src, patch + (u & 1) * ST_PBUF + q * 512);
  };
  auto dma_w = [&](int gs) {
    const int u = gs / 9, tap = gs - u * 9;
    const int slab = slab_of_unit(u);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int piece = wave * 2 + j;
      const int s = piece * 64 + lane;
      const int n = s / ST_CPX, pos = s - n * ST_CPX;
      const int cd = st_wpos(n, pos);
      st_glds16(p.w + (long)n * K + tap * p.Cin + slab * ST_SLAB + cd * 8, wbuf + (gs % ST_WR) * ST_WBUF + piece * 512);
    }
  };

  for (int j = 0; j < ST_PPW; ++j) dma_patch(0, j);
  dma_w(0);
  if (ST_WR == 3 && my_steps > 1) {
    dma_w(1);
    st_wait<2>();
  } else {
    st_wait<0>();
  }
  __builtin_amdgcn_s_barrier();

  const int frow = lane & 15, g = lane >> 4;
  f4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[a][i] = f4{0.f, 0.f, 0.f, 0.f};
  int pbase[4];  // patch pixel of this lane's output pixel for each m-block (tap (1,1) = centre)
  int cur_item_unit = -1;

  for (int gs = 0; gs < my_steps; ++gs) {
    const int u = gs / 9, tap = gs - u * 9;
    const int wahead = gs + ST_WR - 1;                 // the step whose weights are issued now
    const bool issue_w = wahead < my_steps;
    if (issue_w) dma_w(wahead);
    const bool issue_p = tap == 0 && u + 1 < my_units;
    if (issue_p)
      for (int j = 0; j < ST_PPW; ++j) dma_patch(u + 1, j);
    const int tu = u / nsl;
    if (tu != cur_item_unit) {  // new work item: per-lane patch coordinates of its 4 output pixels
      cur_item_unit = tu;
      int bt, q0, sp;
      item_of_unit(u, bt, q0, sp);
      const int r0 = q0 / W;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = min(q0 + mg * 64 + i * 16 + frow, HW - 1);
        const int r = q / W, c = q - r * W;
        pbase[i] = (r - r0 + 1) * PW + c + 1;
      }
    }
    const int dy = tap / 3, dx = tap - dy * 3;
    const int toff = (dy - 1) * PW + (dx - 1);
    const h16* pb = patch + (u & 1) * ST_PBUF;
    const h16* wb = wbuf + (gs % ST_WR) * ST_WBUF;
    {
      const int cd = g;
      h8 xf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pp = pbase[i] + toff;
        xf[i] = *reinterpret_cast<const h8*>(&pb[(pp * ST_CPX + st_ppos(pp, cd)) * 8]);
        if (p.pre_relu) xf[i] = relu8(xf[i]);
      }
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const int n = (ng * 8 + a) * 16 + frow;
        const h8 wf = *reinterpret_cast<const h8*>(&wb[(n * ST_CPX + st_wpos(n, cd)) * 8]);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[a][i] = mfma16(wf, xf[i], acc[a][i]);
      }
    }
    const bool item_end = tap == 8 && (u % nsl) == nsl - 1;
    if (item_end) {
      int bt, q0, sp;
      item_of_unit(u, bt, q0, sp);
      if (p.nsplit > 1) {
        // fp32 partial sums into this split's workspace slice (epilogue in strip_finish_kernel)
        float* wsp = p.ws + (long)sp * p.ws_slice;
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          const int n = (ng * 8 + a) * 16 + g * 4;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int q = q0 + mg * 64 + i * 16 + frow;
            const f4 v = acc[a][i];
            acc[a][i] = f4{0.f, 0.f, 0.f, 0.f};
            if (q < HW) *reinterpret_cast<f4*>(wsp + ((long)bt * HW + q) * ST_N + n) = v;
          }
        }
      } else {
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          const int n = (ng * 8 + a) * 16 + g * 4;
          const f4 bv = p.bias ? *reinterpret_cast<const f4*>(p.bias + n) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int q = q0 + mg * 64 + i * 16 + frow;
            f4 v = acc[a][i] + bv;
            acc[a][i] = f4{0.f, 0.f, 0.f, 0.f};
            if (q >= HW) continue;
            h4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = (h16)(p.relu_out ? fmaxf(v[r], 0.f) : v[r]);
            const long off = ((long)bt * HW + q) * ST_N + n;
            if (p.res) o += *reinterpret_cast<const h4*>(p.res + off);
            if (p.res2) o += *reinterpret_cast<const h4*>(p.res2 + off);
            *reinterpret_cast<h4*>(p.y + off) = o;
          }
        }
      }
      // compiler-visible vmcnt(0) once per work item: without it the loads / stores above stay
      // "pending" across the loop back-edge and hipcc put an s_waitcnt vmcnt(0) before the first VGPR
      // write of every step (draining the weight ring).  It also drains the ring prefetch in flight
      // here (step t+2's weights, and at tap 8 any issued patch pieces): a per-item cost, measured
      // cheaper than the per-step drains it replaces (profiles/r04_ab_strip_wring3.log)
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    {
      // step gs + 1's weights must have landed; newer than them: this step's weights (2 pieces) and
      // the next unit's patch pieces when issued this step (after the weights) or the previous step
      // (tap 1: before this step's weights; they then land by the end of tap 1, 8 steps early)
      const bool p_prev = tap == 1 && u + 1 < my_units;
      if (issue_w) {
        if (issue_p || p_prev) st_wait<ST_PPW + 2>();
        else st_wait<2>();
      } else {
        if (issue_p || p_prev) st_wait<ST_PPW>();
        else st_wait<0>();
      }
    }
    __builtin_amdgcn_s_barrier();
  }
}

// y = fp16([ReLU](sum_s ws[s] + bias)) + res + res2, 4 channels per thread, slices summed in order.
__global__ __launch_bounds__(256) void strip_finish_kernel(const float* __restrict__ ws, int nsplit, long n4,
                                                           const float* __restrict__ bias, int relu_out,
                                                           const h16* __restrict__ res, const h16* __restrict__ res2,
                                                           h16* __restrict__ y) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    f4 v = reinterpret_cast<const f4*>(ws)[i];
    for (int s = 1; s < nsplit; ++s) v += reinterpret_cast<const f4*>(ws)[s * n4 + i];
    if (bias) v += *reinterpret_cast<const f4*>(bias + ((int)i & (ST_N / 4 - 1)) * 4);
    h4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (h16)(relu_out ? fmaxf(v[r], 0.f) : v[r]);
    if (res) o += reinterpret_cast<const h4*>(res)[i];
    if (res2) o += reinterpret_cast<const h4*>(res2)[i];
    reinterpret_cast<h4*>(y)[i] = o;
  }
}

VDA_KNOB(int, g_st_force_split, 0);  // vda_debug_strip_split (tuning build); 0 = automatic

int st_cus() { return vda_cu_count(); }

// Split count for a served shape: minimise rounds x steps-per-item, charging a split its workspace
// round trip (s slices written + read, ~4 TB/s) in units of a ~1.1 us pipeline step.  Only splits whose
// fp32 slices fit `ws_floats` are considered (the caller's workspace; < 0 = unlimited, for the query).
int st_split(int BT, int H, int W, int Cin, long ws_floats) {
  const int nslab = Cin / ST_SLAB;
  const long M = (long)BT * H * W;
  const long nt = (long)BT * ((H * W + ST_M - 1) / ST_M);
  auto fits = [&](int s) { return s == 1 || ws_floats < 0 || (long)s * M * ST_N <= ws_floats; };
  int best = 1;
  double best_cost = 1e30;
  for (int s = 1; s <= 8; s *= 2) {
    if (nslab % s || !fits(s)) continue;
    const long items = nt * s;
    const double rounds = (double)((items + st_cus() - 1) / st_cus());
    const double ws_us = s > 1 ? 2.0 * s * M * ST_N * 4 / 4e12 * 1e6 : 0.0;
    const double cost = rounds * (nslab / s) * 9 + ws_us / 1.1;
    if (cost < best_cost * 0.97) { best_cost = cost; best = s; }
  }
  if (g_st_force_split > 0 && nslab % g_st_force_split == 0 && fits(g_st_force_split)) best = g_st_force_split;
  return best;
}

}  // namespace

#ifdef VDA_TUNING
extern "C" int vda_debug_strip_split(int32_t nsplit) {
  g_st_force_split = nsplit;
  return 0;
}
#endif

bool vda_conv_strip_serves(int W, int Cin, int Cout) {
  return Cout == ST_N && Cin % ST_SLAB == 0 && W <= ST_MAXW && W >= 16;
}

// Bytes of fp32 split workspace the strip conv would use for this shape (0: no split).
long vda_conv_strip_ws_bytes(int BT, int H, int W, int Cin, int Cout) {
  if (!vda_conv_strip_serves(W, Cin, Cout)) return 0;
  const int s = st_split(BT, H, W, Cin, -1);
  return s > 1 ? (long)s * BT * H * W * ST_N * 4 : 0;
}

// Serves 3x3 / s1 / p1 convs with Cout == 256, Cin % 32 == 0, 16 <= W <= 160 (caller checks the
// epilogue: bias, ReLU, res / res2 with row stride Cout).  Returns 1 when the shape is not served.
// `ws` / `ws_bytes`: the caller's fp32 split workspace (may be NULL / 0: no input-channel split).
// Nothing library-global is written, so concurrent calls on different streams with their own
// workspaces are safe.
int vda_conv_strip(const void* x, const void* w, void* y, const float* bias, int relu_out, int pre_relu,
                   const void* res, const void* res2, int BT, int H, int W, int Cin, int Cout, void* ws_ptr,
                   long ws_bytes, hipStream_t st) {
  if (!vda_conv_strip_serves(W, Cin, Cout)) return 1;
  StripParams p{};
  p.x = (const h16*)x; p.w = (const h16*)w; p.y = (h16*)y; p.bias = bias;
  p.res = (const h16*)res; p.res2 = (const h16*)res2;
  p.H = H; p.W = W; p.Cin = Cin; p.pre_relu = pre_relu; p.relu_out = relu_out;
  p.tiles_per_frame = (H * W + ST_M - 1) / ST_M;
  const long nt = (long)BT * p.tiles_per_frame;
  if (nt > 0x7fffffffL / 8) return vda_set_error(-22, "conv: too many tiles");
  p.ntiles = (int)nt;
  const int nslab = Cin / ST_SLAB;
  const long M = (long)BT * H * W;
  const int best = st_split(BT, H, W, Cin, ws_ptr ? ws_bytes / 4 : 0);
  p.nsplit = best;
  p.nsl = nslab / best;
  float* ws = (float*)ws_ptr;
  if (best > 1) {
    p.ws = ws;
    p.ws_slice = M * ST_N;
  }
  const long nitems = nt * best;
  const int grid = (int)(nitems < st_cus() ? nitems : st_cus());
  hipLaunchKernelGGL(strip_conv_kernel, dim3(grid), dim3(512), 0, st, p);
  if (best > 1) {
    const long n4 = M * ST_N / 4;
    const int fg = (int)std::min<long>((n4 + 255) / 256, 4096);
    hipLaunchKernelGGL(strip_finish_kernel, dim3(fg), dim3(256), 0, st, (const float*)ws, best, n4, bias, relu_out,
                       (const h16*)res, (const h16*)res2, (h16*)y);
  }
  VDA_LAUNCH_CHECK();
  return 0;
}
