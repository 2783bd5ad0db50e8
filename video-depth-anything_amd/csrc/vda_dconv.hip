// Depth-head tail conv on the resized output_conv1 map (dpt_temporal.py:92-97, dpt.py:118-124):
//   depth = relu(b2 + sum_j w2[j] * relu(b1[j] + conv3x3_j(U)))      j = 0..31
// U [BT, H, W, C] fp16 (the bilinear resize to the output size is done before, bit-exact to the
// reference's autocast interpolate); the fp32 conv weights as an exact fp16 hi/lo split, 64 MFMA
// rows (0..31 hi, 32..63 lo), both accumulated in fp32.
//
// Shape of the work: N = 64 MFMA rows only, so the LDS bytes per MFMA are set by how many pixels
// each wave multiplies against the whole 64-row W.  Here a wave owns 64 pixels (4 rows of a 16 x 16
// output tile) x all 64 rows: per tap and 32-channel slab 4 X + 4 W ds_read_b128 feed 16 MFMAs (the
// 8-wave halo kernel of vda_depth.hip reads 6 per 8).  Every lane ends up with hi and lo of the same
// 4 channels, so the hi + lo + b1, ReLU and the 32 -> 1 dot are wave-local (two lane-group shuffles).
//
// Blocks of 4 waves (one per SIMD), TWO blocks per CU (78 KiB LDS each): the blocks do not share
// barriers, so one block's barrier wait / DMA issue overlaps the other's MFMAs.  Persistent over
// tiles; the unit of the pipeline is (tile, 32-channel slab), a phase is one kernel row (3 taps,
// 48 MFMAs per wave: a 1-tap phase left the per-phase barrier / wait / issue work at ~2x the MFMA
// time, measured):
//   patch ring 2 x 21 KiB: the 18 x 18-pixel patch of unit u + 1 is issued by LDS-DMA right after
//                          the first barrier of unit u (21 one-KiB pieces, 6 / 5 per wave) and must
//                          land by its last;  slot = pixel * 4 + (chunk ^ ((pixel >> 1) & 3))
//   W ring 3 x 12 KiB:     the 3 x 64 x 32 W slice of phase g + 2 is issued right after barrier g
//                          (3 pieces per wave) into the slot phase g - 1 read;
//                          slot = tap * 256 + row * 4 + (chunk ^ ((row >> 1) & 3))
// one counted vmcnt + one raw s_barrier per phase; inside a phase the fragments of tap t + 1 are
// read while tap t's MFMAs run.  Both layouts are conflict-free for the ds_read_b128 lane groups at
// any tap offset (16 consecutive pixels / rows, chunks c and c + 1).
#include "vda_common.h"
#include "../../include/vda.h"

namespace {

constexpr int DC_T = 16, DC_P = 18;
constexpr int DC_NPIX = DC_P * DC_P;            // 324
constexpr int DC_PP = (DC_NPIX * 4 + 63) / 64;  // 21 one-KiB pieces per patch slot
constexpr int DC_PPW = (DC_PP + 3) / 4;         // per wave, at most (6)
constexpr int DC_PSLOT = DC_PP * 512;           // halfs
constexpr int DC_WROW = 3 * 64 * 32;            // halfs of one phase's W (3 taps x 64 rows x 32 channels)
constexpr int DC_SRCP = 12;                     // UPS: 1-KiB pieces of the source-region slot (192 pixels)
constexpr int DC_SSLOT = DC_SRCP * 512;         // halfs


template <int N>
__device__ __forceinline__ void dc_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void dc_wait_n(int n) {  // n: wave-uniform, 0..9
  if (n >= 9) dc_wait<9>();
  else if (n == 8) dc_wait<8>();
  else if (n == 7) dc_wait<7>();
  else if (n == 6) dc_wait<6>();
  else if (n == 5) dc_wait<5>();
  else if (n == 4) dc_wait<4>();
  else if (n == 3) dc_wait<3>();
  else if (n == 2) dc_wait<2>();
  else if (n == 1) dc_wait<1>();
  else dc_wait<0>();
}
// lgkmcnt(0) as the builtin (vmcnt / expcnt untouched): the compiler then knows the fragments read
// before it are complete and adds no wait of its own for them after later reads
__device__ __forceinline__ void dc_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

// UPS: U is the map BEFORE the bilinear (align_corners=True) resize from (Hs, Ws) to (H, W); each
// unit's patch is interpolated in LDS from a staged source region (bilerp8, the resize kernel's
// formula, separably: bit-identical to resize + conv) by the block's own waves after their MFMAs of the unit's
// middle row, while the other block of the CU keeps the matrix cores busy.  W then uses a 2-slot ring
// (one phase ahead) to make room for the 12-KiB source slot.
#ifdef VDA_TS  // per-block phase-class cycle sums of the fused depth conv (tools/ts_dconv.py; experiments only)
__device__ unsigned long long g_dcts[1024][12];
#endif
template <bool UPS>
__global__ __launch_bounds__(256, 2) void depth_conv_kernel(const h16* __restrict__ U, const h16* __restrict__ w1,
                                                           const float* __restrict__ b1, const float* __restrict__ w2,
                                                           const float* __restrict__ b2, float* __restrict__ depth,
                                                           int H, int W, int C, int tiles_x, int tiles_y, int ntiles,
                                                           int Hs, int Ws, int stagger) {
  constexpr int DC_WRING = UPS ? 2 : 3;
  __shared__ __attribute__((aligned(1024))) h16 sm[2 * DC_PSLOT + DC_WRING * DC_WROW + (UPS ? DC_SSLOT : 0)];
  h16* const psm = sm;
  h16* const wsm = sm + 2 * DC_PSLOT;
  h16* const ssm = sm + 2 * DC_PSLOT + DC_WRING * DC_WROW;  // UPS source region [px][4 chunks]

  int tid;
  asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"((int)threadIdx.x));
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nslab = C / 32;
  const int my_tiles = (int)blockIdx.x < ntiles ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int my_units = my_tiles * nslab;
  if (my_units == 0) return;
  const int G = my_units * 3;                    // phases = kernel rows
  const long K = 9L * C;
  const int my_pp = (DC_PP - 1 - wave) / 4 + 1;  // patch pieces of this wave (6 or 5)

  auto tile_of = [&](int i, int& bt, int& y0, int& x0) {  // i-th tile of this block
    const int t = blockIdx.x + i * gridDim.x;
    const int tx = t % tiles_x, r = t / tiles_x;
    y0 = (r % tiles_y) * DC_T;
    x0 = tx * DC_T;
    bt = r / tiles_y;
  };
  // Per-lane constants, computed once (no per-phase division or 64-bit address math):
  //  patch piece j (q = wave + 4 j): this lane's pixel row / column in the patch and source chunk
  int pmeta[DC_PPW];
#pragma unroll
  for (int j = 0; j < DC_PPW; ++j) {
    const int q = wave + 4 * j;
    const int s = q * 64 + lane;
    const int p = s >> 2;
    const int cd = (s & 3) ^ ((p >> 1) & 3);
    const int pr = p / DC_P;
    pmeta[j] = (q < DC_PP && p < DC_NPIX) ? (pr | ((p - pr * DC_P) << 8) | (cd << 16)) : -1;
  }
  //  W piece j (k = 3 wave + j: tap k / 4, rows 16 (k % 4) ..): byte offset of this lane's 16 B in row
  //  n of w1 for kernel row 0, slab 0 (the row / slab part goes to the scalar soffset)
  unsigned wvo[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int k = wave * 3 + j;
    const int n = (k & 3) * 16 + (lane >> 2);
    const int cd = (lane & 3) ^ ((n >> 1) & 3);
    wvo[j] = (unsigned)((n * (int)K + (k >> 2) * C + cd * 8) * 2);
  }
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)w1, (short)0, (int)(64 * K * 2), 0x00020000);
  const long fr_halfs = UPS ? (long)Hs * Ws * C : (long)H * W * C;
  // this wave's patch pieces of unit u -> patch slot (u & 1); out-of-image pixels read zeros (offset
  // past the frame's records)
  auto patch_dma = [&](int u) {
    int bt, y0, x0;
    tile_of(u / nslab, bt, y0, x0);
    const int slab = u - (u / nslab) * nslab;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(U + bt * fr_halfs), (short)0, (int)(fr_halfs * 2), 0x00020000);
#pragma unroll
    for (int j = 0; j < DC_PPW; ++j) {
      const int q = wave + 4 * j;
      if (q < DC_PP) {
        const int pm = pmeta[j];
        const int py = y0 - 1 + (pm & 0xff), px = x0 - 1 + ((pm >> 8) & 0xff);
        const bool ok = pm >= 0 && (unsigned)py < (unsigned)H && (unsigned)px < (unsigned)W;
        const unsigned vo = ok ? (unsigned)(((py * W + px) * C + ((pm >> 16) & 3) * 8) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (VDA_LDS void*)(psm + (u & 1) * DC_PSLOT + q * 512), 16, (int)vo,
                                                 slab * 64, 0, 0);
      }
    }
  };
  // UPS: source region of unit u's patch: rows sy_lo .. sy_lo + SR - 1, columns sx_lo .. + SC - 1
  const float usy = (UPS && H > 1) ? (float)(Hs - 1) / (float)(H - 1) : 0.f;
  const float usx = (UPS && W > 1) ? (float)(Ws - 1) / (float)(W - 1) : 0.f;
  auto src_region = [&](int y0, int x0, int& sy_lo, int& sx_lo, int& SR, int& SC) {
    sy_lo = (int)(usy * (float)max(y0 - 1, 0));
    sx_lo = (int)(usx * (float)max(x0 - 1, 0));
    SR = min((int)(usy * (float)min(y0 + DC_T, H - 1)) + 1, Hs - 1) - sy_lo + 1;
    SC = min((int)(usx * (float)min(x0 + DC_T, W - 1)) + 1, Ws - 1) - sx_lo + 1;
  };
  // this wave's 3 source pieces (q = 3 wave + j: pixels 16 q .. + 15 of the SR x SC region, 4 chunks
  // each, unswizzled) of unit u -> the source slot
  auto src_dma = [&](int u) {
    int bt, y0, x0, sy_lo, sx_lo, SR, SC;
    tile_of(u / nslab, bt, y0, x0);
    src_region(y0, x0, sy_lo, sx_lo, SR, SC);
    const int slab = u - (u / nslab) * nslab;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(U + bt * fr_halfs), (short)0, (int)(fr_halfs * 2), 0x00020000);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int q = wave * 3 + j;
      const int sl = q * 64 + lane;
      const int px = sl >> 2;
      const int r = px / SC, c = px - r * SC;
      const unsigned vo = r < SR ? (unsigned)((((sy_lo + r) * Ws + sx_lo + c) * C + (sl & 3) * 8) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (VDA_LDS void*)(ssm + q * 512), 16, (int)vo, slab * 64, 0, 0);
    }
  };
  // interpolate unit u's patch from the source slot into patch slot (u & 1) (padding pixels -> 0),
  // separably: bilerp8_mix's blend is o = fma(wy, bot, uy * top) with top / bot the horizontal blends
  // fma(wx, B, ux * A) of source rows sy0 / sy1 at the output column, and a source row's horizontal
  // blend at a column does not depend on the output row that uses it, so each is formed once per
  // (column, source row) and carried down the column: the same ops, bit-identical to bilerp8_mix per
  // pixel (and so to vda_upsample_bilinear), in ~45 % of its VALU.
  // Thread = (column px_l, channel chunk c, 6-row segment): waves 0..2 own columns 0..15 of segment
  // `wave` (the row, hence sy0 / sy1 / wy, is wave-uniform), lanes 0..23 of wave 3 columns 16, 17.
  auto interp_sep = [&](int u) {
    int bt, y0, x0, sy_lo, sx_lo, SR, SC;
    tile_of(u / nslab, bt, y0, x0);
    src_region(y0, x0, sy_lo, sx_lo, SR, SC);
    (void)bt; (void)SR;
    const bool w3 = wave == 3;
    const int seg = w3 ? lane >> 3 : wave;
    const int px_l = w3 ? 16 + ((lane >> 2) & 1) : lane >> 2, c = lane & 3;
    if (w3 && lane >= 24) return;
    const int pxg = x0 - 1 + px_l;
    const bool okx = (unsigned)pxg < (unsigned)W;
    const float ox = (float)min(max(pxg, 0), W - 1);
    const int sx0 = (int)(usx * ox), sx1 = min(sx0 + 1, Ws - 1);
    const float wx = ac_weight(usx, ox, sx0), ux = 1.f - wx;
    const int c0 = sx0 - sx_lo, c1 = sx1 - sx_lo;
    auto hrow = [&](int sy, float (&t)[8]) {
      const int r = (sy - sy_lo) * SC;
      const uint4 a = *reinterpret_cast<const uint4*>(ssm + ((r + c0) * 4 + c) * 8);
      const uint4 b = *reinterpret_cast<const uint4*>(ssm + ((r + c1) * 4 + c) * 8);
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
    for (int k = 0; k < 6; ++k) {
      const int pr = seg * 6 + k;
      const int pyg = y0 - 1 + pr;
      const float oy = (float)min(max(pyg, 0), H - 1);
      const int sy0 = (int)(usy * oy), sy1 = min(sy0 + 1, Hs - 1);
      const float wy = ac_weight(usy, oy, sy0), uy = 1.f - wy;
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
      const uint4 v = ok ? make_uint4(o[0], o[1], o[2], o[3]) : make_uint4(0u, 0u, 0u, 0u);
      const int p = pr * DC_P + px_l;
      *reinterpret_cast<uint4*>(psm + (u & 1) * DC_PSLOT + (p * 4 + (c ^ ((p >> 1) & 3))) * 8) = v;
    }
  };
  // this wave's 3 pieces of phase g's W slice (kernel row dy = g % 3 of unit g / 3) -> slot g % 3
  auto w_dma = [&](int g) {
    const int u = g / 3, dy = g - u * 3;
    const int slab = u % nslab;
    const int so = (dy * 3 * C + slab * 32) * 2;
#pragma unroll
    for (int j = 0; j < 3; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (VDA_LDS void*)(wsm + (g % DC_WRING) * DC_WROW + (wave * 3 + j) * 512),
                                               16, (int)wvo[j], so, 0, 0);
  };

  f4 acc[4][4];
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[n][m] = f4{0.f, 0.f, 0.f, 0.f};

  // start stagger (tuning build, vda_debug_dconv_stagger): the second half of the grid - the second block
  // on each CU - starts `stagger` x 1024 cycles late, so the two blocks' interpolation rows fall out of phase
  if (stagger > 0 && (int)blockIdx.x >= (int)gridDim.x / 2)
    for (int i = 0; i < stagger; ++i) __builtin_amdgcn_s_sleep(16);
  if constexpr (UPS) {
    // prologue: unit 0's source region -> its patch (interpolated), W(0); unit 1's source in flight
    src_dma(0);
    w_dma(0);
    dc_wait<0>();
    __builtin_amdgcn_s_barrier();
    interp_sep(0);
    dc_lgkm0();
    __builtin_amdgcn_s_barrier();
    if (my_units > 1) src_dma(1);
  } else {
    // prologue: unit 0's patch and W(0) retired, W(1) in flight
    patch_dma(0);
    w_dma(0);
    if (G > 1) {
      w_dma(1);
      dc_wait<3>();
    } else {
      dc_wait<0>();
    }
  }

  const int frow = lane & 15, g4 = lane >> 4;
  // epilogue constants: this lane's 4 hi channels g4 * 4 + r of n-blocks 0 and 1
  float bb[2][4], ww[2][4];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bb[n][r] = b1[n * 16 + g4 * 4 + r];
      ww[n][r] = w2[n * 16 + g4 * 4 + r];
    }
  const float bias2 = b2[0];
  // fragment read offsets (halfs): X of patch row wave * 4 + k (k = m + dy, 0..5), column frow + t;
  // W row n * 16 + frow of a slot (tap t adds t * 2048)
  int xo[6][3], wo[4];
#pragma unroll
  for (int k = 0; k < 6; ++k)
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int p = (wave * 4 + k) * DC_P + frow + t;
      xo[k][t] = (p * 4 + (g4 ^ ((p >> 1) & 3))) * 8;
    }
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int row = n * 16 + frow;
    wo[n] = (row * 4 + (g4 ^ ((row >> 1) & 3))) * 8;
  }

  auto read_tap = [&](const h16* ps, const h16* wb, int dy, int t, h8 (&xf)[4], h8 (&wf)[4]) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      int o = xo[m][t];  // dy is wave-uniform: select the row offset without dynamic register indexing
      if (dy == 1) o = xo[m + 1][t];
      if (dy == 2) o = xo[m + 2][t];
      xf[m] = *reinterpret_cast<const h8*>(&ps[o]);
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) wf[n] = *reinterpret_cast<const h8*>(&wb[t * 2048 + wo[n]]);
  };
  auto mfma_tap = [&](const h8 (&xf)[4], const h8 (&wf)[4]) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[n][m] = mfma16(wf[n], xf[m], acc[n][m]);
  };

#ifdef VDA_TS
  // class of the phase that just ended: its row dy (0..2), 3 = a tile's last phase (with the epilogue);
  // sums of s_memtime deltas between phase-start barriers, and of the end-of-phase wait + barrier alone
  unsigned long long tsa[4] = {0, 0, 0, 0}, tsn[4] = {0, 0, 0, 0}, tsw = 0;
  const unsigned long long ts_rt0 = __builtin_amdgcn_s_memrealtime(), ts_c0 = __builtin_amdgcn_s_memtime();
  unsigned long long ts_prev = ts_c0, ts_pre = ts_c0;
  int ts_cls = -1;
#endif
  auto phase = [&](int g, int u, int dy) {
    __builtin_amdgcn_s_barrier();
#ifdef VDA_TS
    {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c == ts_cls) { tsa[c] += now - ts_prev; ++tsn[c]; }
      if (ts_cls >= 0) tsw += now - ts_pre;
      ts_prev = now;
    }
#endif
    // after barrier g every wave is done with phase g - 1's reads: refill its W slot, and (first
    // phase of a unit) the patch slot unit u - 1 read
    const bool wnext = g + (UPS ? 1 : 2) < G;
    if (wnext) w_dma(g + (UPS ? 1 : 2));
    if constexpr (UPS) {
      if (dy == 2 && u + 2 < my_units) src_dma(u + 2);  // the source slot interp_sep(u + 1) read in row 1
    } else {
      if (dy == 0 && u + 1 < my_units) patch_dma(u + 1);
    }
    const h16* ps = psm + (u & 1) * DC_PSLOT;
    const h16* wb = wsm + (g % DC_WRING) * DC_WROW;
    h8 xa[4], wa[4], xb[4], wb2[4];
    read_tap(ps, wb, dy, 0, xa, wa);
    dc_lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    read_tap(ps, wb, dy, 1, xb, wb2);
    __builtin_amdgcn_sched_barrier(0);
    mfma_tap(xa, wa);
    __builtin_amdgcn_sched_barrier(0);
    dc_lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    read_tap(ps, wb, dy, 2, xa, wa);
    __builtin_amdgcn_sched_barrier(0);
    mfma_tap(xb, wb2);
    __builtin_amdgcn_sched_barrier(0);
    dc_lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    mfma_tap(xa, wa);
    __builtin_amdgcn_sched_barrier(0);
    return wnext;
  };

  for (int u = 0; u < my_units; ++u) {
#pragma unroll
   for (int dy = 0; dy < 3; ++dy) {
    const int g = u * 3 + dy;
    const bool wnext = phase(g, u, dy);
    if (dy == 2 && (u % nslab) == nslab - 1) {
      // tile done: hi + lo + b1 -> ReLU -> . w2 over this lane's 8 channels, then the 4 lane groups
      int bt, y0, x0;
      tile_of(u / nslab, bt, y0, x0);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        float part = 0.f;
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r) part += fmaxf(acc[n][m][r] + acc[n + 2][m][r] + bb[n][r], 0.f) * ww[n][r];
        part += __shfl_xor(part, 16, 64);
        part += __shfl_xor(part, 32, 64);
        const int y = y0 + wave * 4 + m, x = x0 + frow;
        if (lane < 16 && y < H && x < W) depth[((long)bt * H + y) * W + x] = fmaxf(part + bias2, 0.f);
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[n][m] = f4{0.f, 0.f, 0.f, 0.f};
      }
    }
#ifdef VDA_TS
    ts_cls = (dy == 2 && (u % nslab) == nslab - 1) ? 3 : dy;
#endif
    if constexpr (UPS) {
      // row 1: this unit's MFMAs are issued; build the next unit's patch (its source region arrived
      // by the row-0 wait), writes complete before barrier g + 1 (a 3 + 3 split over rows 1 and 2,
      // with the source staged in row 0, measured 3 % slower: the source fetch then has one phase)
      if (dy == 1 && u + 1 < my_units) {
        interp_sep(u + 1);
        dc_lgkm0();
      }
      // W(g + 1) (issued this phase) must have landed before barrier g + 1; so must, at row 0, the
      // source region of unit u + 1 (issued in row 2 of unit u - 1).  Newer: row 2's source pieces
#ifdef VDA_TS
      ts_pre = __builtin_amdgcn_s_memtime();
#endif
      dc_wait_n(dy == 2 && u + 2 < my_units ? 3 : 0);
    } else {
      // W(g + 1) (issued in phase g - 1) and, at a unit's last row, the next unit's patch (issued in its
      // first row, after that row's W pieces) must have landed before barrier g + 1.  Newer than
      // W(g + 1): this phase's 3 W pieces and, in rows 0 and 1, the patch pieces of row 0
      dc_wait_n((wnext ? 3 : 0) + (dy <= 1 && u + 1 < my_units ? my_pp : 0));
    }
   }
  }
#ifdef VDA_TS
  if (UPS && threadIdx.x == 0 && blockIdx.x < 1024) {
    for (int c = 0; c < 4; ++c) { g_dcts[blockIdx.x][c] = tsa[c]; g_dcts[blockIdx.x][4 + c] = tsn[c]; }
    g_dcts[blockIdx.x][8] = __builtin_amdgcn_s_memrealtime() - ts_rt0;
    g_dcts[blockIdx.x][9] = __builtin_amdgcn_s_memtime() - ts_c0;
    g_dcts[blockIdx.x][10] = tsw;
  }
#endif
}

}  // namespace

#ifdef VDA_TS
extern "C" int vda_debug_dconv_timestamps(void* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dcts), sizeof(g_dcts), 0, hipMemcpyDeviceToHost);
}
#endif

// vda_debug_dconv (tuning build): -1 automatic (fused), 0 never, 2 resize + unfused depth conv
VDA_KNOB(int, g_dconv_mode, -1);
VDA_KNOB(int, g_dconv_stagger, 0);  // vda_debug_dconv_stagger

bool vda_depth_conv_serves(int H, int W, int C) { return C % 32 == 0 && C > 0 && H > 0 && W > 0 && g_dconv_mode != 0; }

// depth tail on the already-resized map U [BT, H, W, C] (C % 32 == 0).  Returns 1 when not served.
int vda_depth_conv(const void* U, const void* w1, const float* b1, const float* w2, const float* b2, float* depth,
                   int BT, int H, int W, int C, hipStream_t st) {
  if (!vda_depth_conv_serves(H, W, C)) return 1;
  const int cus = vda_cu_count();
  const int tiles_x = (W + DC_T - 1) / DC_T, tiles_y = (H + DC_T - 1) / DC_T;
  const long nt = (long)BT * tiles_x * tiles_y;
  if (nt > 0x7fffffffL / 9 / ((C + 31) / 32)) return vda_set_error(-22, "depth conv: too many tiles");
  const int ntiles = (int)nt;
  const int grid = ntiles < 2 * cus ? ntiles : 2 * cus;
  hipLaunchKernelGGL(depth_conv_kernel<false>, dim3(grid), dim3(256), 0, st, (const h16*)U, (const h16*)w1, b1, w2, b2,
                     depth, H, W, C, tiles_x, tiles_y, ntiles, H, W, 0);
  VDA_LAUNCH_CHECK();
  return 0;
}

// the same on the UN-resized map x [BT, Hs, Ws, C] (Hs <= H, Ws <= W): the bilinear resize is computed
// while each patch is built (bit-identical to vda_upsample_bilinear + vda_depth_conv); the staged
// source region of a tile (<= floor(17 * scale) + 3 pixels per side) must fit 192 pixels.
bool vda_depth_conv_fused_serves(int Hs, int Ws, int H, int W, int C) {
  if (!vda_depth_conv_serves(H, W, C) || g_dconv_mode == 2 || Hs > H || Ws > W || Hs < 1 || Ws < 1) return false;
  const float sy = H > 1 ? (float)(Hs - 1) / (float)(H - 1) : 0.f, sx = W > 1 ? (float)(Ws - 1) / (float)(W - 1) : 0.f;
  return ((int)(17.f * sy) + 3) * ((int)(17.f * sx) + 3) <= 192;
}

int vda_depth_conv_fused(const void* x, const void* w1, const float* b1, const float* w2, const float* b2,
                         float* depth, int BT, int Hs, int Ws, int H, int W, int C, hipStream_t st) {
  if (!vda_depth_conv_fused_serves(Hs, Ws, H, W, C)) return 1;
  const int cus = vda_cu_count();
  const int tiles_x = (W + DC_T - 1) / DC_T, tiles_y = (H + DC_T - 1) / DC_T;
  const long nt = (long)BT * tiles_x * tiles_y;
  if (nt > 0x7fffffffL / 9 / ((C + 31) / 32)) return vda_set_error(-22, "depth conv: too many tiles");
  const int ntiles = (int)nt;
  const int grid = ntiles < 2 * cus ? ntiles : 2 * cus;
  hipLaunchKernelGGL(depth_conv_kernel<true>, dim3(grid), dim3(256), 0, st, (const h16*)x, (const h16*)w1, b1, w2, b2,
                     depth, H, W, C, tiles_x, tiles_y, ntiles, Hs, Ws, (int)g_dconv_stagger);
  VDA_LAUNCH_CHECK();
  return 0;
}

#ifdef VDA_TUNING
extern "C" int vda_debug_dconv(int32_t mode) {
  g_dconv_mode = mode;
  return 0;
}
extern "C" int vda_debug_dconv_stagger(int32_t units1024) {
  g_dconv_stagger = units1024;
  return 0;
}
#endif
