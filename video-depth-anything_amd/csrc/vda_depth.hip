// Depth-head tail as a halo-tiled conv (dpt_temporal.py:92-99, dpt.py:118-124, video_depth.py:63-64):
//   depth = relu(b2 + sum_j w2[j] * relu(b1[j] + conv3x3_j(U)))      j = 0..31
// over U = the (already resized) output_conv1 map [BT, H, W, C] fp16, with the fp32 conv weights as an
// exact fp16 hi/lo split (64 MFMA output rows: 32 hi, 32 lo; both accumulate in fp32).
//
// Why a halo tile: the implicit-GEMM conv re-reads every input pixel once per tap (9x) and reloads the
// 147-KB weight tile for every 256-pixel tile; with only 64 output rows the kernel was L2->LDS bound
// (~360 TF/s).  Here a block owns a 16x16 output tile and stages the 18x18-pixel input patch ONCE per
// 64-channel slab (LDS-DMA, 41.5 KB), then runs all 9 taps out of LDS: input traffic 1.27x the map
// instead of 9x, weights streamed per (slab, kernel row) step (24 KB: 3 taps) from L2.
//
// Block = 8 waves, persistent over tiles.  Wave w: output rows 4*(w&3) .. +3 of the tile (4 m-blocks of
// 16 pixels) x n-blocks {ng, ng+2} (ng = w>>2): hi and lo rows of the same 16 output channels, so the
// hi+lo sum, +b1, ReLU and the w2 dot are wave-local; the two ng halves meet in a 1-KB LDS scratch.
// Pipeline: 2 patch slabs (ring) and 2 weight steps (ring); per step (one kernel row: 48 MFMAs per
// wave) each wave issues the next step's weight pieces, and on a unit's first step the whole next
// patch slab; the counted end-of-step vmcnt leaves only those patch pieces in flight; one raw
// s_barrier per step.  LDS layouts: patch slot = pixel*CPX + (chunk ^ (pixel & 7)) (CPX = 8 chunks of
// 16 B) resp. ^((pixel >> 1) & 3) (CPX = 4); weights row*CPX + (chunk ^ ((row >> 1) & (CPX-1))):
// conflict-free for the ds_read_b128 lane groups at any patch offset (brute-forced).
#include "vda_common.h"
#include "../../include/vda.h"

namespace {

__device__ __attribute__((aligned(64))) uint4 g_dz_page[4];

constexpr int DT = 16;              // output tile edge
constexpr int DP = DT + 2;          // patch edge (halo 1)
constexpr int DNPIX = DP * DP;      // 324

__device__ __forceinline__ void dh_glds16(const void* src, h16* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (VDA_LDS void*)lds_base, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void dh_wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int CPX>
__device__ __forceinline__ int patch_pos(int p, int cd) {
  if constexpr (CPX == 8) return cd ^ (p & 7);
  else return cd ^ ((p >> 1) & 3);
}
template <int CPX>
__device__ __forceinline__ int w_pos(int n, int cd) {
  return cd ^ ((n >> 1) & (CPX - 1));
}

// DEPTH: the depth tail (64 weight rows = 32 hi + 32 lo, wave n-blocks {ng, ng+2}, ReLU/1x1/ReLU epilogue
// to fp32 depth).  !DEPTH: a plain 3x3 conv with NROW output channels (wave n-blocks ng*NB4 .. +NB4-1,
// epilogue +bias [ReLU] -> fp16 NHWC).  TPS taps per pipeline step (3 = one kernel row, or 1).
template <int SLAB, int NROW, int TPS, bool DEPTH>
__global__ __launch_bounds__(512) void halo_conv_kernel(const h16* __restrict__ U, const h16* __restrict__ w1,
                                                        const float* __restrict__ b1, const float* __restrict__ w2,
                                                        const float* __restrict__ b2, float* __restrict__ depth,
                                                        h16* __restrict__ yout, int relu_out,
                                                        int H, int W, int C, int tiles_x, int tiles_y, int ntiles) {
  static_assert(!DEPTH || NROW == 64, "depth tail: 64 weight rows");
  constexpr int NB = NROW / 32;                          // n-blocks per wave (2 for the depth tail)
  constexpr int CPX = SLAB / 8;                          // 16-B chunks per pixel per slab
  constexpr int PSLOT = DNPIX * CPX;                     // 16-B slots of one patch slab
  constexpr int PP = (PSLOT + 63) / 64;                  // 1-KiB DMA pieces per slab
  constexpr int PBUF = PP * 64 * 8;                      // halfs per patch ring slot
  constexpr int WROW = TPS * CPX;                        // slots per weight row per step
  constexpr int WSLOT = NROW * WROW;                     // 16-B slots of one weight step
  constexpr int WBUF = WSLOT * 8;                        // halfs
  constexpr int WPCS = WSLOT / 64;                       // weight pieces per step (24 or 12)
  constexpr int WPW = (WPCS + 7) / 8;                    // per wave (3 or 2; surplus waves duplicate)
  constexpr int ND = SLAB / 32;                          // MFMA k-depths per tap
  __shared__ __attribute__((aligned(16))) h16 dsm[2 * PBUF + 2 * WBUF + 512];
  h16* patch = dsm;                                      // [2][PBUF]
  h16* wbuf = dsm + 2 * PBUF;                            // [2][WBUF]
  float* scratch = reinterpret_cast<float*>(dsm + 2 * PBUF + 2 * WBUF);  // [256]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mg = wave & 3, ng = wave >> 2;
  const int nslab = C / SLAB;
  const int K = 9 * C;
  const int units_per_tile = nslab;
  constexpr int SPU = 9 / TPS;                           // steps per unit (slab)
  // tiles of this block: t = blockIdx.x + i * gridDim.x
  const int my_tiles = blockIdx.x < ntiles ? (ntiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  const int my_units = my_tiles * units_per_tile;
  if (my_units == 0) return;
  const int my_steps = my_units * SPU;
  const void* zero = (const void*)g_dz_page;

  auto tile_of_unit = [&](int u, int& bt, int& y0, int& x0) {
    const int t = blockIdx.x + (u / units_per_tile) * gridDim.x;
    const int tx = t % tiles_x;
    const int r = t / tiles_x;
    const int ty = r % tiles_y;
    bt = r / tiles_y;
    y0 = ty * DT;
    x0 = tx * DT;
  };
  // piece q of unit u's patch slab -> ring slot (u & 1)
  auto dma_patch = [&](int u, int q) {
    int bt, y0, x0;
    tile_of_unit(u, bt, y0, x0);
    const int slab = u % units_per_tile;
    const int s = q * 64 + lane;
    const int p = s / CPX, pos = s - p * CPX;
    const int cd = patch_pos<CPX>(p, pos);
    const int pr = p / DP;
    const int py = y0 - 1 + pr, px = x0 - 1 + (p - pr * DP);
    const void* src = zero;
    if (p < DNPIX && (unsigned)py < (unsigned)H && (unsigned)px < (unsigned)W)
      src = U + (((long)bt * H + py) * W + px) * C + slab * SLAB + cd * 8;
    dh_glds16(src, patch + (u & 1) * PBUF + q * 512);
  };
  // weight pieces of global step gs (kernel row dy of slab) -> ring slot (gs & 1)
  auto dma_w = [&](int gs) {
    const int u = gs / SPU, st = gs - u * SPU;
    const int slab = u % units_per_tile;
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int piece = (wave * WPW + j) % WPCS;
      const int s = piece * 64 + lane;
      const int n = s / WROW, rem = s - n * WROW;
      const int tt = rem / CPX, pos = rem - tt * CPX;
      const int cd = w_pos<CPX>(n, pos);
      dh_glds16(w1 + (long)n * K + (st * TPS + tt) * C + slab * SLAB + cd * 8, wbuf + (gs & 1) * WBUF + piece * 512);
    }
  };

  // prologue: patch of unit 0 (all pieces, split over waves) + weights of step 0
  for (int q = wave; q < PP; q += 8) dma_patch(0, q);
  dma_w(0);
  dh_wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();

  const int frow = lane & 15, g = lane >> 4;
  const int jh = ng * 16 + g * 4;                        // this lane's 4 output channels (hi rows)
  f4 acc[NB][4];
#pragma unroll
  for (int a = 0; a < NB; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[a][i] = f4{0.f, 0.f, 0.f, 0.f};
  const int my_pp = (PP - 1 - wave) / 8 + 1;             // next-slab patch pieces of this wave
  constexpr int PPMAX = (PP + 7) / 8;
  float pend[4] = {0.f, 0.f, 0.f, 0.f};
  int pend_bt = -1, pend_y0 = 0, pend_x0 = 0;

  for (int gs = 0; gs < my_steps; ++gs) {
    const int u = gs / SPU, st = gs - u * SPU;
    // weights of the next step first, then (first step of a unit) the whole next patch slab: the
    // end-of-step wait then leaves exactly the patch pieces in flight, and they land by the end of
    // the unit's second step
    if (gs + 1 < my_steps) dma_w(gs + 1);
    const bool issue_p = st == 0 && u + 1 < my_units;
    if (issue_p)
      for (int j = 0; j < my_pp; ++j) dma_patch(u + 1, wave + j * 8);
    // ---- TPS taps x ND k-depths x (NB x 4) MFMAs
    const h16* pb = patch + (u & 1) * PBUF;
    const h16* wb = wbuf + (gs & 1) * WBUF;
#pragma unroll
    for (int tt = 0; tt < TPS; ++tt) {
      const int tap = st * TPS + tt;
      const int dy = tap / 3, dx = tap - dy * 3;
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const int cd = d * 4 + g;
        h8 wf[NB], xf[4];
#pragma unroll
        for (int a = 0; a < NB; ++a) {
          const int n = (DEPTH ? ng + 2 * a : ng * NB + a) * 16 + frow;
          wf[a] = *reinterpret_cast<const h8*>(&wb[(n * WROW + tt * CPX + w_pos<CPX>(n, cd)) * 8]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int p = (mg * 4 + i + dy) * DP + frow + dx;
          xf[i] = *reinterpret_cast<const h8*>(&pb[(p * CPX + patch_pos<CPX>(p, cd)) * 8]);
        }
#pragma unroll
        for (int a = 0; a < NB; ++a)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[a][i] = mfma16(wf[a], xf[i], acc[a][i]);
      }
    }
    const bool tile_end = st == SPU - 1 && (u % units_per_tile) == units_per_tile - 1;
    if (!DEPTH && tile_end) {
      // +bias [ReLU] -> fp16 NHWC; lane: 4 consecutive channels of pixel (row mg*4+i, col frow)
      int bt, y0, x0;
      tile_of_unit(u, bt, y0, x0);
#pragma unroll
      for (int a = 0; a < NB; ++a) {
        const int n = (ng * NB + a) * 16 + g * 4;
        const f4 bv = b1 ? *reinterpret_cast<const f4*>(b1 + n) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int y = y0 + mg * 4 + i, x = x0 + frow;
          f4 v = acc[a][i] + bv;
          h4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (h16)(relu_out ? fmaxf(v[r], 0.f) : v[r]);
          if (y < H && x < W) *reinterpret_cast<h4*>(yout + (((long)bt * H + y) * W + x) * NROW + n) = o;
          acc[a][i] = f4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
    if (DEPTH && tile_end) {
      // hi + lo + b1 -> ReLU -> * w2 over this lane's 4 channels, then the 4 lane groups
      float bb[4], ww[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) { bb[r] = b1[jh + r]; ww[r] = w2[jh + r]; }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float part = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) part += fmaxf(acc[0][i][r] + acc[NB - 1][i][r] + bb[r], 0.f) * ww[r];
        part += __shfl_xor(part, 16, 64);
        part += __shfl_xor(part, 32, 64);
        pend[i] = part;
#pragma unroll
        for (int a = 0; a < NB; ++a) acc[a][i] = f4{0.f, 0.f, 0.f, 0.f};
      }
      if (ng == 1 && lane < 16) {
#pragma unroll
        for (int i = 0; i < 4; ++i) scratch[(mg * 4 + i) * 16 + lane] = pend[i];
      }
      tile_of_unit(u, pend_bt, pend_y0, pend_x0);
    }
    if (issue_p) {
      if (my_pp == PPMAX) dh_wait_vmcnt<PPMAX>();
      else dh_wait_vmcnt<PPMAX - 1>();
    } else {
      dh_wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (DEPTH && tile_end) {
      if (ng == 0 && lane < 16) {
        const float bias2 = b2[0];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int y = pend_y0 + mg * 4 + i, x = pend_x0 + lane;
          const float v = pend[i] + scratch[(mg * 4 + i) * 16 + lane] + bias2;
          if (y < H && x < W) depth[((long)pend_bt * H + y) * W + x] = fmaxf(v, 0.f);
        }
      }
    }
  }
}

int g_num_cus = 0;

}  // namespace

// called by vda_depth_head (vda_gemm.hip) after the resize into ws; returns 1 if the shape is not
// supported here (caller falls back to the implicit-GEMM kernel)
int vda_depth_halo(const void* U, const void* w1, const float* b1, const float* w2, const float* b2, float* depth,
                   int BT, int H, int W, int C, hipStream_t st) {
  if (!(C == 32 || C % 64 == 0)) return 1;
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    g_num_cus = n > 0 ? n : 256;
  }
  const int tiles_x = (W + DT - 1) / DT, tiles_y = (H + DT - 1) / DT;
  const long nt = (long)BT * tiles_x * tiles_y;
  if (nt > 0x7fffffffL) return vda_set_error(-22, "depth head: too many tiles");
  const int ntiles = (int)nt;
  const int grid = ntiles < g_num_cus ? ntiles : g_num_cus;
  if (C == 32)
    hipLaunchKernelGGL((halo_conv_kernel<32, 64, 3, true>), dim3(grid), dim3(512), 0, st, (const h16*)U, (const h16*)w1,
                       b1, w2, b2, depth, (h16*)nullptr, 0, H, W, C, tiles_x, tiles_y, ntiles);
  else
    hipLaunchKernelGGL((halo_conv_kernel<64, 64, 3, true>), dim3(grid), dim3(512), 0, st, (const h16*)U, (const h16*)w1,
                       b1, w2, b2, depth, (h16*)nullptr, 0, H, W, C, tiles_x, tiles_y, ntiles);
  VDA_LAUNCH_CHECK();
  return 0;
}

// 3x3 / stride 1 / pad 1 conv, Cin % 64 == 0, Cout == 128, epilogue +bias [ReLU] (output_conv1,
// dpt.py:117, at 296^2): the halo tile cuts the 9x implicit-GEMM input re-read.  Returns 1 when the
// shape is not one this kernel serves (caller uses the implicit-GEMM conv).
int vda_conv_halo(const void* x, const void* w, void* y, const float* bias, int relu, int BT, int H, int W, int Cin,
                  int Cout, hipStream_t st) {
  if (Cout != 128 || Cin % 64 != 0) return 1;
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    g_num_cus = n > 0 ? n : 256;
  }
  const int tiles_x = (W + DT - 1) / DT, tiles_y = (H + DT - 1) / DT;
  const long nt = (long)BT * tiles_x * tiles_y;
  if (nt > 0x7fffffffL) return vda_set_error(-22, "conv: too many tiles");
  const int ntiles = (int)nt;
  const int grid = ntiles < g_num_cus ? ntiles : g_num_cus;
  hipLaunchKernelGGL((halo_conv_kernel<64, 128, 1, false>), dim3(grid), dim3(512), 0, st, (const h16*)x, (const h16*)w,
                     bias, (const float*)nullptr, (const float*)nullptr, (float*)nullptr, (h16*)y, relu, H, W, Cin,
                     tiles_x, tiles_y, ntiles);
  VDA_LAUNCH_CHECK();
  return 0;
}
