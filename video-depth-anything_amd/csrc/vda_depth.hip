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
#ifdef VDA_TS  // per-block step-class cycle sums of output_conv1 (tools/ts_oc1.py; experiments only)
__device__ unsigned long long g_dts[1024][24];
#endif

constexpr int DT = 16;              // output tile edge
constexpr int DP = DT + 2;          // patch edge (halo 1)
constexpr int DNPIX = DP * DP;      // 324

__device__ __forceinline__ void dh_glds16(const void* src, h16* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (VDA_LDS void*)lds_base, 16, 0, 0);
}
typedef unsigned dh_u4 __attribute__((ext_vector_type(4)));
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
// align_corners=True source coordinate, as vda_upsample_bilinear computes it (torch upsample_bilinear2d);
// sc = (in - 1) / (out - 1) (0 for out == 1) is hoisted out by the caller, same float division
__device__ __forceinline__ float dh_ac_scale(int in, int out) {
  return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
}
__device__ __forceinline__ void dh_ac_coord(int o, int in, float sc, int& i0, int& i1, float& w) {
  const float f = sc * (float)o;
  i0 = (int)f;
  i1 = min(i0 + 1, in - 1);
  w = ac_weight(sc, (float)o, i0);
}

// DEPTH: the depth tail (64 weight rows = 32 hi + 32 lo, wave n-blocks {ng, ng+2}, ReLU/1x1/ReLU epilogue
// to fp32 depth).  !DEPTH: a plain 3x3 conv with NROW output channels (wave n-blocks ng*NB4 .. +NB4-1,
// epilogue +bias [ReLU] -> fp16 NHWC).  TPS taps per pipeline step (3 = one kernel row, or 1).
// UPS: U is the [BT, Hs, Ws, C] map BEFORE the bilinear (align_corners=True) resize to (H, W), and the
// patch is interpolated instead of copied, so the resized map is never written to HBM.  The source
// region a tile's 18x18 patch needs (<= 12 x 12 pixels for a scale <= 0.6) is staged ONCE per slab by
// LDS-DMA in place of the patch (same fixed-count piece scheme, 3 pieces per wave, one slot: it is
// filled at a unit's first step and consumed at its last), and at the unit's last step every thread
// interpolates its 16-B patch slots from LDS in fp32 (bilerp8: the resize kernel's formula and
// op order, so the fp16 values are bit-identical) into the other patch ring slot.
// IW (UPS only): IW extra interpolation waves (8 .. 8+IW-1) own the source staging and the
// interpolation: they fetch unit u+1's source region at steps 0-1 of unit u and build its patch over the
// following steps (ups_interp_item, 64 IW items a step), beside the 8 MFMA waves' taps, which then never
// stop for the interpolation; every wave takes every step barrier.
template <int SLAB, int NROW, int TPS, bool DEPTH, bool UPS = false, int IW = 0>
__global__ __launch_bounds__(512 + 64 * IW) void halo_conv_kernel(const h16* __restrict__ U, const h16* __restrict__ w1,
                                                        const float* __restrict__ b1, const float* __restrict__ w2,
                                                        const float* __restrict__ b2, float* __restrict__ depth,
                                                        h16* __restrict__ yout, int relu_out,
                                                        int H, int W, int C, int tiles_x, int tiles_y, int ntiles,
                                                        int Hs = 0, int Ws = 0) {
  static_assert(!DEPTH || NROW == 64, "depth tail: 64 weight rows");
  constexpr int NB = NROW / 32;                          // n-blocks per wave (2 for the depth tail)
  constexpr int CPX = SLAB / 8;                          // 16-B chunks per pixel per slab
  // LIN (the plain conv): the patch is linear in the pixel with the pixel stride padded to PSTR slots
  // (10 for 64-channel slabs, 6 for 32: conflict-free for the ds_read_b128 lane groups at any pixel
  // offset, brute-forced), so a tap moves every fragment read by one constant: per step the reads
  // cost one address add per output row and the rest are immediates.  The depth-tail instantiations
  // keep the XOR-swizzled dense layout (their LDS has no room for the padding).
  constexpr bool LIN = !DEPTH;
  constexpr int PSTR = LIN ? (CPX == 8 ? 10 : 6) : CPX;  // 16-B slots per patch pixel
  constexpr int PSLOT = DNPIX * PSTR;                    // 16-B slots of one patch slab
  constexpr int PP = (PSLOT + 63) / 64;                  // 1-KiB DMA pieces per slab
  constexpr int PBUF = (UPS ? PSLOT : PP * 64) * 8;      // halfs per patch ring slot
  constexpr int WROW = TPS * CPX;                        // slots per weight row per step
  constexpr int WSLOT = NROW * WROW;                     // 16-B slots of one weight step
  constexpr int WBUF = WSLOT * 8;                        // halfs
  constexpr int WPCS = WSLOT / 64;                       // weight pieces per step (24 or 12)
  constexpr int WPW = (WPCS + 7) / 8;                    // per wave (3 or 2; surplus waves duplicate)
  constexpr int ND = SLAB / 32;                          // MFMA k-depths per tap
  constexpr int WRING = 2;                               // weight ring
  static_assert(!UPS || 9 / TPS >= 2, "UPS: >= 2 steps per unit");
  static_assert(IW == 0 || (UPS && TPS == 1), "interpolation waves: the 9-step fused-resize conv");
  constexpr int SPPW = (192 * CPX + 511) / 512;          // UPS source pieces per wave (fixed count)
  constexpr int SSLOT = UPS ? SPPW * 8 * 64 : 0;         // source slots: >= 192 pixels x CPX chunks
  __shared__ __attribute__((aligned(16))) h16 dsm[2 * PBUF + WRING * WBUF + SSLOT * 8 + 512];
  h16* patch = dsm;                                      // [2][PBUF]
  h16* wbuf = dsm + 2 * PBUF;                            // [WRING][WBUF]
  h16* sbuf = dsm + 2 * PBUF + WRING * WBUF;             // [SSLOT * 8] (UPS)
  float* scratch = reinterpret_cast<float*>(dsm + 2 * PBUF + WRING * WBUF + SSLOT * 8);  // [256]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mg = wave & 3, ng = wave >> 2;
  const bool iwave = IW > 0 && wave >= 8;                // interpolation wave (no MFMA work)
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

  // a unit's coordinates are formed once (the divisions are scalar but long), not per DMA piece
  struct Ud { int bt, y0, x0, slab, sy_lo, sx_lo, SR, SC; };
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
  auto dma_patch = [&](int u, const Ud& ud, int q) {
    const int bt = ud.bt, y0 = ud.y0, x0 = ud.x0, slab = ud.slab;
    const int s = q * 64 + lane;
    const int p = s / PSTR, pos = s - p * PSTR;
    const int cd = LIN ? pos : patch_pos<CPX>(p, pos);
    const int pr = p / DP;
    const int py = y0 - 1 + pr, px = x0 - 1 + (p - pr * DP);
    const void* src = zero;
    if (p < DNPIX && pos < CPX && (unsigned)py < (unsigned)H && (unsigned)px < (unsigned)W)
      src = U + (((long)bt * H + py) * W + px) * C + slab * SLAB + cd * 8;
    dh_glds16(src, patch + (u & 1) * PBUF + q * 512);
  };
  // weight pieces of global step gs (kernel row dy of slab) -> ring slot (gs & 1)
  // UPS: source region of unit u's patch: rows sy_lo .. sy_lo + SR - 1, columns sx_lo .. + SC - 1
  constexpr int USL = DNPIX * CPX;                       // 16-B patch slots read by the taps
  constexpr int UCH = UPS ? (USL + 511) / 512 : 1;       // patch slots per thread
  const float usy = UPS ? dh_ac_scale(Hs, H) : 0.f, usx = UPS ? dh_ac_scale(Ws, W) : 0.f;
  auto src_region = [&](int y0, int x0, int& sy_lo, int& sx_lo, int& SR, int& SC) {
    sy_lo = (int)(usy * (float)max(y0 - 1, 0));
    sx_lo = (int)(usx * (float)max(x0 - 1, 0));
    SR = min((int)(usy * (float)min(y0 + DT, H - 1)) + 1, Hs - 1) - sy_lo + 1;
    SC = min((int)(usx * (float)min(x0 + DT, W - 1)) + 1, Ws - 1) - sx_lo + 1;
  };
  auto make_ud = [&](int u) {
    Ud ud;
    tile_of_unit(u, ud.bt, ud.y0, ud.x0);
    ud.slab = u % units_per_tile;
    ud.sy_lo = ud.sx_lo = ud.SR = ud.SC = 0;
    if constexpr (UPS) src_region(ud.y0, ud.x0, ud.sy_lo, ud.sx_lo, ud.SR, ud.SC);
    return ud;
  };
  // piece j (of SPPW) of unit u's source region -> sbuf; slot = pixel * CPX + chunk
  auto dma_src = [&](const Ud& ud, int q) {
    const int bt = ud.bt, sy_lo = ud.sy_lo, sx_lo = ud.sx_lo, SR = ud.SR, SC = ud.SC, slab = ud.slab;
    const int s = q * 64 + lane;
    const int px = s / CPX, cd = s % CPX;
    const int r = px / SC, c = px - r * SC;
    const void* src = zero;
    if (r < SR) src = U + (((long)bt * Hs + sy_lo + r) * Ws + sx_lo + c) * C + slab * SLAB + cd * 8;
    dh_glds16(src, sbuf + q * 512);
  };
  // interpolate unit u's patch from sbuf into patch ring slot (u & 1); padding pixels -> 0
  // slots t0 + k * tstride (k < NK) of the patch (t0 = this thread's first)
  auto ups_interp = [&](int u, const Ud& ud, int t0, int tstride, auto nk_tag) {
    constexpr int NK = decltype(nk_tag)::value;
    const int y0 = ud.y0, x0 = ud.x0, sy_lo = ud.sy_lo, sx_lo = ud.sx_lo, SC = ud.SC;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int s = t0 + k * tstride;
      const int sc = min(s, USL - 1);
      const int p = sc / CPX, pos = sc - p * CPX;
      const int cd = LIN ? pos : patch_pos<CPX>(p, pos);
      const int pr = p / DP;
      const int py = y0 - 1 + pr, px = x0 - 1 + (p - pr * DP);
      const bool ok = (unsigned)py < (unsigned)H && (unsigned)px < (unsigned)W;
      int sy0, sy1, sx0, sx1;
      float wy, wx;
      dh_ac_coord(min(max(py, 0), H - 1), Hs, usy, sy0, sy1, wy);
      dh_ac_coord(min(max(px, 0), W - 1), Ws, usx, sx0, sx1, wx);
      const int r0 = (sy0 - sy_lo) * SC, r1 = (sy1 - sy_lo) * SC, c0 = sx0 - sx_lo, c1 = sx1 - sx_lo;
      const h8 a = *reinterpret_cast<const h8*>(sbuf + ((r0 + c0) * CPX + cd) * 8);
      const h8 b = *reinterpret_cast<const h8*>(sbuf + ((r0 + c1) * CPX + cd) * 8);
      const h8 c = *reinterpret_cast<const h8*>(sbuf + ((r1 + c0) * CPX + cd) * 8);
      const h8 d = *reinterpret_cast<const h8*>(sbuf + ((r1 + c1) * CPX + cd) * 8);
      const h8 v = bilerp8(a, b, c, d, wx, wy);
      const uint4 z = make_uint4(0u, 0u, 0u, 0u);
      const uint4 o = ok ? __builtin_bit_cast(uint4, v) : z;
      const int slot = LIN ? p * PSTR + pos : s;
      // asm store: a compiler-visible LDS store that may alias the LDS-DMA ring gets an s_waitcnt
      // vmcnt(0) in front of it, which drained the next step's weight DMA before the interpolation
      if (s < USL)
        asm volatile("ds_write_b128 %0, %1" ::"v"((unsigned)(uintptr_t)(VDA_LDS h16*)(patch + (u & 1) * PBUF + slot * 8)),
                     "v"(__builtin_bit_cast(dh_u4, o))
                     : "memory");
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the stores above are invisible to the compiler's counts
  };
  // The interpolation waves' form of ups_interp (LIN layout): item = (patch column, channel chunk,
  // 6-row segment).  The blend is o = fma(wy, bot, uy * top) with top / bot the horizontal blends
  // fma(wx, B, ux * A) of source rows sy0 / sy1 at the column; a source row's horizontal blend at a
  // column does not depend on the output row that uses it, so it is formed once per (column, source
  // row) and carried down the segment: per pixel the ops of bilerp8_mix (bit-identical to bilerp8, the
  // resize kernel's blend) in about half its VALU.
  constexpr int ISEG = 3;                                // rows per item (6: 1809, 9: 1966 vs 1781 us)
  constexpr int NITEM = (DP / ISEG) * DP * CPX;          // 432 for a 64-channel slab
  auto ups_interp_item = [&](int u, const Ud& ud, int it) {
    if (it >= NITEM) return;
    const int y0 = ud.y0, x0 = ud.x0, sy_lo = ud.sy_lo, sx_lo = ud.sx_lo, SC = ud.SC;
    const int cd = it % CPX, col = (it / CPX) % DP, seg = it / (CPX * DP);
    const int pxg = x0 - 1 + col;
    const bool okx = (unsigned)pxg < (unsigned)W;
    int sx0, sx1;
    float wx;
    dh_ac_coord(min(max(pxg, 0), W - 1), Ws, usx, sx0, sx1, wx);
    const float ux = 1.f - wx;
    const int c0 = sx0 - sx_lo, c1 = sx1 - sx_lo;
    auto hrow = [&](int sy, float (&t)[8]) {
      const int r = (sy - sy_lo) * SC;
      const uint4 a = *reinterpret_cast<const uint4*>(sbuf + ((r + c0) * CPX + cd) * 8);
      const uint4 b = *reinterpret_cast<const uint4*>(sbuf + ((r + c1) * CPX + cd) * 8);
      const unsigned A[4] = {a.x, a.y, a.z, a.w}, B[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t[2 * j] = fma_mix_lo(wx, B[j], fma_mix_lo(ux, A[j], -0.f));
        t[2 * j + 1] = fma_mix_hi(wx, B[j], fma_mix_hi(ux, A[j], -0.f));
      }
    };
    float top[8], bot[8];
    int s0 = -1, s1 = -1;
#pragma unroll
    for (int k = 0; k < ISEG; ++k) {
      const int pr = seg * ISEG + k;
      const int pyg = y0 - 1 + pr;
      int sy0, sy1;
      float wy;
      dh_ac_coord(min(max(pyg, 0), H - 1), Hs, usy, sy0, sy1, wy);
      const float uy = 1.f - wy;
      if (sy0 != s0) {  // scale <= 1: the source rows advance by at most one per output row
        if (sy0 == s1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) top[e] = bot[e];
        } else {
          hrow(sy0, top);
        }
        hrow(sy1, bot);
        s0 = sy0;
        s1 = sy1;
      }
      unsigned o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float ol = fma_f32(wy, bot[2 * j], mul_f32(uy, top[2 * j]));
        const float oh = fma_f32(wy, bot[2 * j + 1], mul_f32(uy, top[2 * j + 1]));
        typedef float f2v __attribute__((ext_vector_type(2)));
        o[j] = __builtin_bit_cast(unsigned, __builtin_convertvector(f2v{ol, oh}, h2));
      }
      const bool ok = okx && (unsigned)pyg < (unsigned)H;
      const dh_u4 v = ok ? dh_u4{o[0], o[1], o[2], o[3]} : dh_u4{0u, 0u, 0u, 0u};
      const int slot = (pr * DP + col) * PSTR + cd;
      asm volatile("ds_write_b128 %0, %1" ::"v"((unsigned)(uintptr_t)(VDA_LDS h16*)(patch + (u & 1) * PBUF + slot * 8)),
                   "v"(v)
                   : "memory");
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the asm stores are invisible to the compiler's counts
  };
  // weight pieces of step st of a unit of slab `slab` -> ring slot `wslot`
  auto dma_w = [&](int st, int slab, int wslot) {
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int piece = (wave * WPW + j) % WPCS;
      const int s = piece * 64 + lane;
      const int n = s / WROW, rem = s - n * WROW;
      const int tt = rem / CPX, pos = rem - tt * CPX;
      const int cd = w_pos<CPX>(n, pos);
      dh_glds16(w1 + (long)n * K + (st * TPS + tt) * C + slab * SLAB + cd * 8, wbuf + wslot * WBUF + piece * 512);
    }
  };

  // prologue: patch of unit 0 (all pieces, split over waves) + weights of step 0
  Ud ud_next = make_ud(0);
  if constexpr (UPS) {
    if (!iwave) {
      for (int j = 0; j < SPPW; ++j) dma_src(ud_next, wave + j * 8);
      dma_w(0, ud_next.slab, 0);
    }
    dh_wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (!iwave) ups_interp(0, ud_next, tid, 512, std::integral_constant<int, UCH>{});
    __syncthreads();  // patch slot 0 written, source slot free for unit 1
  } else {
    for (int q = wave; q < PP; q += 8) dma_patch(0, ud_next, q);
    dma_w(0, ud_next.slab, 0);
    dh_wait_vmcnt<0>();
  }
  __builtin_amdgcn_s_barrier();

  if constexpr (IW > 0) {
    if (iwave) {
      // the interpolation waves' own step loop (same barrier sequence as the MFMA waves' loop below, no
      // accumulators live): unit u+1's source region in two halves at steps 0 and 1 (waited for before
      // step 2's barrier; all at step 0 and blending from step 2: 1820 vs 1784 us), its patch items over
      // steps 3 .. 2 + ISTEPS (64 IW a step); the step barriers publish the writes
      constexpr int SPI = SPPW * 8 / IW;                 // source pieces per interpolation wave
      constexpr int ISTEPS = (NITEM + 64 * IW - 1) / (64 * IW);
      static_assert(LIN && SPPW * 8 % IW == 0 && ISTEPS <= SPU - 3, "interpolation wave split");
      int iu = 0, ist = 0;
      for (int gs = 0; gs < my_steps; ++gs) {
        if (ist == 0 && iu + 1 < my_units) {
          ud_next = make_ud(iu + 1);
          for (int j = 0; j < SPI / 2; ++j) dma_src(ud_next, (wave - 8) + j * IW);
        }
        if (ist == 1 && iu + 1 < my_units)
          for (int j = SPI / 2; j < SPI; ++j) dma_src(ud_next, (wave - 8) + j * IW);
        if (ist >= 3 && ist < 3 + ISTEPS && iu + 1 < my_units)
          ups_interp_item(iu + 1, ud_next, (ist - 3) * 64 * IW + (tid - 512));
        if (ist == 2) dh_wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        if (++ist == SPU) {
          ist = 0;
          ++iu;
        }
      }
      return;
    }
  }
  const int frow = lane & 15, g = lane >> 4;
  const int jh = ng * 16 + g * 4;                        // this lane's 4 output channels (hi rows)
  // LIN: lane-constant byte offsets of the fragment reads (output row i, k-depth d and the tap are
  // immediates / one scalar per step); W rows keep their XOR swizzle, which depends on the row only
  const unsigned lin_x = (unsigned)(((mg * 4) * DP + frow) * PSTR + g) * 16u;
  unsigned lin_w[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    const int n0r = (DEPTH ? ng : ng * NB) * 16 + frow;
    lin_w[d] = (unsigned)(n0r * WROW + w_pos<CPX>(n0r, d * 4 + g)) * 16u;
  }
  f4 acc[NB][4];
#pragma unroll
  for (int a = 0; a < NB; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[a][i] = f4{0.f, 0.f, 0.f, 0.f};
  // the plain conv's bias, held for the whole launch (a lane's channels do not change with the tile): a
  // load in the epilogue made every tile end wait (vmcnt(0)) for it
  f4 bias_r[DEPTH ? 1 : NB];
#pragma unroll
  for (int a = 0; a < (DEPTH ? 1 : NB); ++a)
    bias_r[a] = (!DEPTH && b1) ? *reinterpret_cast<const f4*>(b1 + (ng * NB + a) * 16 + g * 4) : f4{0.f, 0.f, 0.f, 0.f};
  const int my_pp = (PP - 1 - wave) / 8 + 1;             // next-slab patch pieces of this wave
  constexpr int PPMAX = (PP + 7) / 8;
  float pend[4] = {0.f, 0.f, 0.f, 0.f};
  int pend_bt = -1, pend_y0 = 0, pend_x0 = 0;

  // step counters kept incrementally (no per-step division): unit u, its step st and slab
  int u = 0, st = 0, slab = 0;
#ifdef VDA_TS
  // class = step within the unit (0..SPU-1), SPU = a tile's last step; sums of s_memtime deltas between
  // consecutive end-of-step barriers (and of the end-of-step wait + barrier alone), taken by every wave
  // (uniform), stored by thread 0 at the end
  unsigned long long tsa[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned tsn[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long ts_rt0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long ts_c0 = __builtin_amdgcn_s_memtime();
  unsigned long long ts_prev = ts_c0, tsw = 0;
#endif
  for (int gs = 0; gs < my_steps; ++gs) {
    // weights of the next step first, then (first step of a unit) the whole next patch slab: the
    // end-of-step wait then leaves exactly the patch pieces in flight, and they land by the end of
    // the unit's second step
    const bool issue_p = st == 0 && u + 1 < my_units;
    if (issue_p) ud_next = make_ud(u + 1);
    if (gs + 1 < my_steps) {
      if (st + 1 < SPU) dma_w(st + 1, slab, (gs + 1) & 1);
      else dma_w(0, slab + 1 == nslab ? 0 : slab + 1, (gs + 1) & 1);
    }
    if constexpr (UPS) {
      // first step: the next unit's source region (lands by the end of the second step); last step:
      // interpolate the next unit's patch from it into the other patch slot (published by this
      // step's barrier; the source slot is refilled only after it)
      if constexpr (IW == 0) {
        if (issue_p)
          for (int j = 0; j < SPPW; ++j) dma_src(ud_next, wave + j * 8);
        if (st == SPU - 1 && u + 1 < my_units) ups_interp(u + 1, ud_next, tid, 512, std::integral_constant<int, UCH>{});
      }
    } else if (issue_p) {
      for (int j = 0; j < my_pp; ++j) dma_patch(u + 1, ud_next, wave + j * 8);
    }
    // ---- TPS taps x ND k-depths x (NB x 4) MFMAs
    const h16* pb = patch + (u & 1) * PBUF;
    const h16* wb = wbuf + (gs & 1) * WBUF;
    if constexpr (LIN) {
      // one scalar per step: patch slot + this step's first tap offset, W slot (opaque: no strength
      // reduction of the modulo counters into per-read VALU)
      const int tap0 = st * TPS;
      unsigned xs, ws;
      asm volatile("s_mov_b32 %0, %1" : "=s"(xs)
                   : "s"((unsigned)((u & 1) * PBUF * 2 + ((tap0 / 3) * DP + (tap0 % 3)) * PSTR * 16)));
      asm volatile("s_mov_b32 %0, %1" : "=s"(ws) : "s"((unsigned)((gs & 1) * WBUF * 2)));
      const char* pxb = reinterpret_cast<const char*>(patch) + xs + lin_x;
      const char* wxb[ND];
#pragma unroll
      for (int d = 0; d < ND; ++d) wxb[d] = reinterpret_cast<const char*>(wbuf) + ws + lin_w[d];
#pragma unroll
      for (int tt = 0; tt < TPS; ++tt) {  // taps of one step share the kernel row (TPS 3) or are one
#pragma unroll
        for (int d = 0; d < ND; ++d) {
          h8 wf[NB], xf[4];
#pragma unroll
          for (int a = 0; a < NB; ++a)
            wf[a] = *reinterpret_cast<const h8*>(wxb[d] + ((DEPTH ? 2 * a : a) * 16 * WROW + tt * CPX) * 16);
#pragma unroll
          for (int i = 0; i < 4; ++i)
            xf[i] = *reinterpret_cast<const h8*>(pxb + (i * DP + tt) * PSTR * 16 + d * 64);
#pragma unroll
          for (int a = 0; a < NB; ++a)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[a][i] = mfma16(wf[a], xf[i], acc[a][i]);
        }
      }
    } else {
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
    }
    const bool tile_end = st == SPU - 1 && slab == units_per_tile - 1;
    if (!DEPTH && tile_end) {
      // +bias [ReLU] -> fp16 NHWC.  A lane holds 4 consecutive channels of pixel (row mg*4+i, col frow)
      // per n-block; lane groups g and g^1 (lanes l, l^16) trade one n-block of each pair so that every
      // lane stores 8 consecutive channels (16 B: half the store instructions of 8-B pieces).  Buffer
      // stores over the frame, pixels outside the map dropped by the range check, so every lane issues
      // exactly NB / 2 * 4 of them (the end-of-step wait below counts them).
      int bt, y0, x0;
      tile_of_unit(u, bt, y0, x0);
      const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(yout + (long)bt * H * W * NROW), (short)0, (int)((long)H * W * NROW * 2), 0x00020000);
      const bool godd = (g & 1) != 0;
#pragma unroll
      for (int a = 0; a < NB; a += 2) {
        const f4 bv0 = bias_r[DEPTH ? 0 : a], bv1 = bias_r[DEPTH ? 0 : a + 1];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int y = y0 + mg * 4 + i, x = x0 + frow;
          const f4 v0 = acc[a][i] + bv0, v1 = acc[a + 1][i] + bv1;
          h4 o0, o1;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            o0[r] = (h16)(relu_out ? fmaxf(v0[r], 0.f) : v0[r]);
            o1[r] = (h16)(relu_out ? fmaxf(v1[r], 0.f) : v1[r]);
          }
          const uint2 u0 = __builtin_bit_cast(uint2, o0), u1 = __builtin_bit_cast(uint2, o1);
          const uint2 snd = godd ? u0 : u1;
          float ax, bx, ay, by;
          swap16_pair(__builtin_bit_cast(float, snd.x), ax, bx);
          swap16_pair(__builtin_bit_cast(float, snd.y), ay, by);
          const uint2 rcv = make_uint2(__builtin_bit_cast(unsigned, godd ? ax : bx), __builtin_bit_cast(unsigned, godd ? ay : by));
          const u32x4 val = godd ? u32x4{rcv.x, rcv.y, u1.x, u1.y} : u32x4{u0.x, u0.y, rcv.x, rcv.y};
          const int n = (ng * NB + a + (godd ? 1 : 0)) * 16 + (g & 2) * 4;
          const unsigned vo = (y < H && x < W) ? (unsigned)(((y * W + x) * NROW + n) * 2) : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b128(val, ys, vo, 0, 0);
          acc[a][i] = f4{0.f, 0.f, 0.f, 0.f};
          acc[a + 1][i] = f4{0.f, 0.f, 0.f, 0.f};
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
#ifdef VDA_TS
    const unsigned long long ts_pre = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (UPS) {
      if (IW == 0 && issue_p) dh_wait_vmcnt<SPPW>();
      else if (IW > 0 && tile_end) dh_wait_vmcnt<NB / 2 * 4>();  // the next step's weights, not the tile's stores
      else dh_wait_vmcnt<0>();
    } else if (issue_p) {
      if (my_pp == PPMAX) dh_wait_vmcnt<PPMAX>();
      else dh_wait_vmcnt<PPMAX - 1>();
    } else {
      dh_wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
#ifdef VDA_TS
    {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      const int cls = tile_end ? SPU : st;
#pragma unroll
      for (int c = 0; c <= SPU && c < 10; ++c)
        if (c == cls) { tsa[c] += now - ts_prev; ++tsn[c]; }
      tsw += now - ts_pre;
      ts_prev = now;
    }
#endif
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
    if (++st == SPU) {
      st = 0;
      ++u;
      if (++slab == nslab) slab = 0;
    }
  }
#ifdef VDA_TS
  if (!DEPTH && UPS && tid == 0 && blockIdx.x < 1024) {
    const unsigned long long rt = __builtin_amdgcn_s_memrealtime() - ts_rt0, cy = __builtin_amdgcn_s_memtime() - ts_c0;
    for (int c = 0; c < 10; ++c) { g_dts[blockIdx.x][c] = tsa[c]; g_dts[blockIdx.x][10 + c] = tsn[c]; }
    g_dts[blockIdx.x][20] = rt;
    g_dts[blockIdx.x][21] = cy;
    g_dts[blockIdx.x][22] = tsw;
  }
#endif
}

}  // namespace

#ifdef VDA_TS
extern "C" int vda_debug_oc1_timestamps(void* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dts), sizeof(g_dts), 0, hipMemcpyDeviceToHost);
}
#endif

// called by vda_depth_head (vda_gemm.hip) after the resize into ws; returns 1 if the shape is not
// supported here (caller falls back to the implicit-GEMM kernel)
int vda_depth_halo(const void* U, const void* w1, const float* b1, const float* w2, const float* b2, float* depth,
                   int BT, int H, int W, int C, hipStream_t st) {
  if (!(C == 32 || C % 64 == 0)) return 1;
  const int cus = vda_cu_count();
  const int tiles_x = (W + DT - 1) / DT, tiles_y = (H + DT - 1) / DT;
  const long nt = (long)BT * tiles_x * tiles_y;
  if (nt > 0x7fffffffL) return vda_set_error(-22, "depth head: too many tiles");
  const int ntiles = (int)nt;
  const int grid = ntiles < cus ? ntiles : cus;
  if (C == 32)
    hipLaunchKernelGGL((halo_conv_kernel<32, 64, 3, true>), dim3(grid), dim3(512), 0, st, (const h16*)U, (const h16*)w1,
                       b1, w2, b2, depth, (h16*)nullptr, 0, H, W, C, tiles_x, tiles_y, ntiles);
  else
    hipLaunchKernelGGL((halo_conv_kernel<64, 64, 3, true>), dim3(grid), dim3(512), 0, st, (const h16*)U, (const h16*)w1,
                       b1, w2, b2, depth, (h16*)nullptr, 0, H, W, C, tiles_x, tiles_y, ntiles);
  VDA_LAUNCH_CHECK();
  return 0;
}

// Depth tail straight from the UN-resized output_conv1 map x [BT, Hs, Ws, C] (C % 64 == 0, Hs <= H,
// Ws <= W): the bilinear resize is computed while the halo patch is built (UPS), so the resized map
// (2.2 GB at ViT-L 32x518^2) is never written.  Returns 1 when the shape is not served.
bool vda_depth_halo_fused_serves(int Hs, int Ws, int H, int W, int C) {
  if (C % 64 != 0 || Hs > H || Ws > W || Hs < 1 || Ws < 1) return false;
  // the staged source region of a tile (<= floor(17 * scale) + 2 rows / columns) must fit 192 pixels
  const float sy = H > 1 ? (float)(Hs - 1) / (float)(H - 1) : 0.f, sx = W > 1 ? (float)(Ws - 1) / (float)(W - 1) : 0.f;
  return ((int)(17.f * sy) + 3) * ((int)(17.f * sx) + 3) <= 192;
}

int vda_depth_halo_fused(const void* x, const void* w1, const float* b1, const float* w2, const float* b2,
                         float* depth, int BT, int Hs, int Ws, int H, int W, int C, hipStream_t st) {
  if (!vda_depth_halo_fused_serves(Hs, Ws, H, W, C)) return 1;
  const int cus = vda_cu_count();
  const int tiles_x = (W + DT - 1) / DT, tiles_y = (H + DT - 1) / DT;
  const long nt = (long)BT * tiles_x * tiles_y;
  if (nt > 0x7fffffffL) return vda_set_error(-22, "depth head: too many tiles");
  const int ntiles = (int)nt;
  const int grid = ntiles < cus ? ntiles : cus;
  hipLaunchKernelGGL((halo_conv_kernel<64, 64, 3, true, true>), dim3(grid), dim3(512), 0, st, (const h16*)x,
                     (const h16*)w1, b1, w2, b2, depth, (h16*)nullptr, 0, H, W, C, tiles_x, tiles_y, ntiles, Hs, Ws);
  VDA_LAUNCH_CHECK();
  return 0;
}

// output_conv1 on the 2x resize of refinenet1's output without writing the resized map: the halo conv
// below with the resize fused into its patch staging (UPS).  x [BT, Hs, Ws, Cin] is the map BEFORE the
// bilinear (align_corners=True) resize to (H, W).  Returns 1 when the shape is not served.
int vda_conv_halo_fused(const void* x, const void* w, void* y, const float* bias, int relu, int BT, int Hs, int Ws,
                        int H, int W, int Cin, int Cout, hipStream_t st) {
  if (Cout != 128 || Cin % 64 != 0 || Hs > H || Ws > W || Hs < 1 || Ws < 1) return 1;
  if ((long)H * W * Cout * 2 >= (1L << 31)) return 1;  // the epilogue's per-frame buffer stores take 32-bit offsets
  const float sy = H > 1 ? (float)(Hs - 1) / (float)(H - 1) : 0.f, sx = W > 1 ? (float)(Ws - 1) / (float)(W - 1) : 0.f;
  if (((int)(17.f * sy) + 3) * ((int)(17.f * sx) + 3) > 192) return 1;
  const int cus = vda_cu_count();
  const int tiles_x = (W + DT - 1) / DT, tiles_y = (H + DT - 1) / DT;
  const long nt = (long)BT * tiles_x * tiles_y;
  if (nt > 0x7fffffffL) return vda_set_error(-22, "conv: too many tiles");
  const int ntiles = (int)nt;
  const int grid = ntiles < cus ? ntiles : cus;
  // 4 interpolation waves (1 / 2: 2571 / 2080 vs 1801 us, profiles/r05_ab_oc1_interp_waves_dconv_separable.log)
  hipLaunchKernelGGL((halo_conv_kernel<64, 128, 1, false, true, 4>), dim3(grid), dim3(768), 0, st, (const h16*)x,
                     (const h16*)w, bias, (const float*)nullptr, (const float*)nullptr, (float*)nullptr, (h16*)y, relu,
                     H, W, Cin, tiles_x, tiles_y, ntiles, Hs, Ws);
  VDA_LAUNCH_CHECK();
  return 0;
}

// 3x3 / stride 1 / pad 1 conv, Cin % 64 == 0, Cout == 128, epilogue +bias [ReLU] (output_conv1,
// dpt.py:117, at 296^2): the halo tile cuts the 9x implicit-GEMM input re-read.  Returns 1 when the
// shape is not one this kernel serves (caller uses the implicit-GEMM conv).
int vda_conv_halo(const void* x, const void* w, void* y, const float* bias, int relu, int BT, int H, int W, int Cin,
                  int Cout, hipStream_t st) {
  if (Cout != 128 || Cin % 64 != 0) return 1;
  if ((long)H * W * Cout * 2 >= (1L << 31)) return 1;  // the epilogue's per-frame buffer stores take 32-bit offsets
  const int cus = vda_cu_count();
  const int tiles_x = (W + DT - 1) / DT, tiles_y = (H + DT - 1) / DT;
  const long nt = (long)BT * tiles_x * tiles_y;
  if (nt > 0x7fffffffL) return vda_set_error(-22, "conv: too many tiles");
  const int ntiles = (int)nt;
  const int grid = ntiles < cus ? ntiles : cus;
  hipLaunchKernelGGL((halo_conv_kernel<64, 128, 1, false>), dim3(grid), dim3(512), 0, st, (const h16*)x, (const h16*)w,
                     bias, (const float*)nullptr, (const float*)nullptr, (float*)nullptr, (h16*)y, relu, H, W, Cin,
                     tiles_x, tiles_y, ntiles);
  VDA_LAUNCH_CHECK();
  return 0;
}
