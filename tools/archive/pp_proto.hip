// Ping-pong GEMM prototype (tuning tool, not product code): two 4-wave groups per 512-thread block
// alternate 256x128 tiles; while one group runs its MFMA main loop over an R-deep ring of BK=32 LDS
// stages, the other group runs the previous tile's epilogue.  Standalone: hipcc -O3 --offload-arch=gfx950
// tools/pp_proto.hip -o build/pp_proto && build/pp_proto
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#include <type_traits>

typedef _Float16 h16;
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#define VDA_LDS __attribute__((address_space(3)))
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace pp {
constexpr int BK = 32, BM = 256, BN = 128;
constexpr int STAGE = (BM + BN) * BK;  // halfs per stage (24 KiB)
constexpr int PPW = 6;                 // DMA pieces (1 KiB) per active wave per stage

__device__ __forceinline__ f4 mfma16(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

template <int N> __device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
template <int N> __device__ __forceinline__ void wait_lgkm() {
  static_assert(N >= 0 && N < 16, "lgkmcnt");
  __builtin_amdgcn_s_waitcnt(0xC07F | (N << 8));
}
// lane id from a volatile mbcnt: lane-derived values are recomputed where used instead of being hoisted
// (and kept live, or spilled) across the persistent tile loop
__device__ __forceinline__ int vlane() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
__device__ __forceinline__ void perm16_swap(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}

__device__ __forceinline__ void tile_coords(int bid, int nwg, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  constexpr int GROUP_M = 8;
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - group * per_group;
  tm = first_m + in_group % gsize;
  tn = in_group / gsize;
}

struct Params {
  const h16* x; const h16* w; h16* y; const float* bias;
  int M, N, K;  // ldx = K, ldy = N
};

// Epilogue of one 16-row block j of a wave tile: bias, fp16, permlane regroup, two 16-B stores of whole
// 128-B lines (as vda_gemm.hip's register epilogue).
__device__ __forceinline__ void epi_j(const Params& p, const f4 (&acc)[4][8], int j, int m0, int n0, int wm, int wn,
                                      __amdgpu_buffer_rsrc_t ry) {
  const int lane = vlane();
  const int mcol = lane & 15, g = lane >> 4;
  f4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = acc[i][j];
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
    o[pp] = u32x4{__builtin_bit_cast(unsigned, h0), __builtin_bit_cast(unsigned, h1), __builtin_bit_cast(unsigned, h2_),
                  __builtin_bit_cast(unsigned, h3)};
  }
  const bool lo8 = (mcol & 8) == 0;
  u32x4 A, B;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const unsigned snd = lo8 ? o[1][k] : o[0][k];
    const unsigned got = (unsigned)__builtin_amdgcn_mov_dpp((int)snd, 0x128, 0xF, 0xF, true);
    A[k] = lo8 ? o[0][k] : got;
    B[k] = lo8 ? got : o[1][k];
  }
  // columns of this lane's two pieces: n0 + wn*64 + 32*pp + 16*(g&1) + 8*(g>>1)
  const int col0 = n0 + wn * 64 + 16 * (g & 1) + 8 * (g >> 1);
  const int col = col0 + (lo8 ? 0 : 32);
  const unsigned cofs = col < p.N ? (unsigned)(col * 2) : 0x80000000u;
  const unsigned vo = (unsigned)((mcol & 7) * p.N * 2) + cofs;  // row offsets of the 16-row block in soffset
  const int so = (wm * 128 + j * 16) * p.N * 2;
  __builtin_amdgcn_raw_buffer_store_b128(A, ry, vo, so, 0);
  __builtin_amdgcn_raw_buffer_store_b128(B, ry, vo, so + 8 * p.N * 2, 0);
}

template <int R>
__global__ __launch_bounds__(512) void pp_gemm(Params p, int tiles_m, int tiles_n) {
  static_assert(R >= 4, "ring depth");
  __shared__ __attribute__((aligned(1024))) h16 smem[R * STAGE];
  const int ntiles = tiles_m * tiles_n;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int grp = wave >> 2, gw = wave & 3;
  const int wm = gw & 1, wn = gw >> 1;
  const int Q = ntiles > (int)blockIdx.x ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int nk = p.K / BK;
  const int total = Q * nk;  // stages of this block

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)((long)p.M * p.K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)((long)p.N * p.K * 2), 0x00020000);

  // DMA lane geometry: piece = 16 rows x 64 B, lane -> local row lane >> 2, physical chunk lane & 3,
  // logical chunk = phys ^ g(row bits 2-3) with g(q) = -q & 3 (conflict-free b128 fragment reads)
  // fragment read lane offset (halfs) within a 16-row block: row frow, logical chunk fchunk
  auto foff_of = [](int lane) {
    const int frow = lane & 15, fchunk = lane >> 4;
    return frow * BK + ((fchunk ^ (-(frow >> 2) & 3)) << 3);
  };

  // per-tile DMA voffsets (bytes) of this wave's 6 pieces (valid only while this wave's group is active)
  unsigned voff[PPW];
  auto set_tile_dma = [&](int q, unsigned (&vo)[PPW]) {
    const int vb = (int)blockIdx.x + q * (int)gridDim.x;
    int tm, tn;
    tile_coords(vb, ntiles, tiles_m, tiles_n, tm, tn);
    const int lane = vlane();
    const int dlr = lane >> 2;
    const int dlc = ((lane & 3) ^ (-(dlr >> 2) & 3)) * 8;  // logical k offset (halfs)
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pi = gw + 4 * i;
      if (i < 4) {
        const int m = tm * BM + pi * 16 + dlr;
        vo[i] = m < p.M ? (unsigned)(((long)m * p.K + dlc) * 2) : 0x80000000u;
      } else {
        const int n = tn * BN + (pi - 16) * 16 + dlr;
        vo[i] = n < p.N ? (unsigned)(((long)n * p.K + dlc) * 2) : 0x80000000u;
      }
    }
  };
  // issue this wave's pieces of block-stage s (tile s / nk, k-step s % nk) into ring slot s % R
  auto issue = [&](int s) {
    const int kk = s % nk;  // voff: those of tile s / nk
    h16* sb = smem + (s % R) * STAGE;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pi = gw + 4 * i;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 4 ? xrs : wrs, (VDA_LDS void*)(sb + pi * 512), 16,
                                               (int)voff[i], kk * BK * 2, 0, 0);
    }
  };

  h8 xf[8], wf[4];
  auto read_x = [&](int s, int j, int fo) {
    xf[j] = *reinterpret_cast<const h8*>(smem + (s % R) * STAGE + fo + (wm * 128 + j * 16) * BK);
  };
  auto read_w = [&](int s, int fo) {
    const h16* sb = smem + (s % R) * STAGE + fo;
#pragma unroll
    for (int i = 0; i < 4; ++i) wf[i] = *reinterpret_cast<const h8*>(sb + (BM + wn * 64 + i * 16) * BK);
  };
  auto read_frags = [&](int s) {
    const int fo = foff_of(vlane());
    read_w(s, fo);
#pragma unroll
    for (int j = 0; j < 8; ++j) read_x(s, j, fo);
  };
  f4 acc[4][8];

  // prologue: group 0 issues stages 0 .. R-2 of its first tile (tile 0 = this block's first tile)
  // NOTE: stages are consecutive per tile; a tile's first R-1 stages may belong to tile 1 when nk < R-1
  // (not supported: nk >= R)
  if (Q == 0) return;
  if (grp == 0) {
    set_tile_dma(0, voff);
    for (int s = 0; s < R - 1 && s < total; ++s) issue(s);
    wait_vm<(R - 2) * PPW>();
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 0) read_frags(0);

  int ep_m0 = 0, ep_n0 = 0;  // coordinates of the tile this group's epilogue handles
  __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void*)p.y, (short)0, 0, 0x00020000);

  for (int q = 0; q < Q; ++q) {
    const bool active = (q & 1) == grp;
    if (active) {
      // DMA coordinates: the active group issues stages s + R - 1, which cross into tile q + 1 in the last
      // R - 1 iterations (tile q + 1 belongs to the OTHER group but the active group issues its pieces)
      if (q > 0) set_tile_dma(q, voff);
      const int fo = foff_of(vlane());
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
      // one K step: wait for my pieces of stage s + 1, barrier, DMA of stage s + R - 1, W fragments of s + 1,
      // the 32 MFMAs of stage s with the X fragments of s + 1 read behind their last use
      auto kstep = [&](int kk, auto hc, auto rc) {
        constexpr int h = decltype(hc)::value;
        constexpr bool rd = decltype(rc)::value;
        const int s = q * nk + kk;
        wait_vm<(R - 3) * PPW>();
        __builtin_amdgcn_s_barrier();
        if (s + R - 1 < total) issue(s + R - 1);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][j] = mfma16(wf[i], xf[j], acc[i][j]);
          if (rd) read_x(s + 1, j, fo);
        }
        if (rd) read_w(s + 1, fo);  // W of s + 1 lands under the next barrier
        __builtin_amdgcn_s_setprio(0);
      };
      using I0 = std::integral_constant<int, 0>;
      using I1 = std::integral_constant<int, 1>;
      using BT = std::integral_constant<bool, true>;
      using BF = std::integral_constant<bool, false>;
      static_assert(R == 5, "tail written for R = 5");
      for (int k = 0; k < nk - 4; k += 2) {
        kstep(k, I0{}, BT{});
        kstep(k + 1, I1{}, BT{});
      }
      set_tile_dma(q + 1, voff);  // from here on the DMA fetches the next tile's first stages
      kstep(nk - 4, I0{}, BT{});
      kstep(nk - 3, I1{}, BT{});
      kstep(nk - 2, I0{}, BT{});
      kstep(nk - 1, I1{}, BF{});
      // this tile's epilogue runs during the next tile (or after the loop)
      const int vb = (int)blockIdx.x + q * (int)gridDim.x;
      int tm, tn;
      tile_coords(vb, ntiles, tiles_m, tiles_n, tm, tn);
      ep_m0 = tm * BM;
      ep_n0 = tn * BN;
      const long mrows = p.M - ep_m0;
      ry = __builtin_amdgcn_make_buffer_rsrc((void*)(p.y + (long)ep_m0 * p.N), (short)0,
                                             (int)(mrows * p.N * 2 < 0x7fffffffL ? mrows * p.N * 2 : 0x7fffffffL), 0x00020000);
    } else {
      // inactive: the previous tile's epilogue in 8 chunks between the active group's barriers
      int kk = 0;
      if (q >= 1) {
        // pieces of stages q*nk + 1 .. q*nk + R - 2 were issued by this group during tile q - 1
        static_assert(R == 5, "wait ladder written for R = 5");
        wait_vm<2 * PPW>(); __builtin_amdgcn_s_barrier();
        wait_vm<1 * PPW>(); __builtin_amdgcn_s_barrier();
        wait_vm<0>(); __builtin_amdgcn_s_barrier();
        kk = 3;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __builtin_amdgcn_s_barrier();
          epi_j(p, acc, j, ep_m0, ep_n0, wm, wn, ry);
        }
        kk = 11;
      }
      for (; kk < nk - 1; ++kk) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_s_barrier();
      if (q + 1 < Q) read_frags((q + 1) * nk);
    }
  }
  // the last tile's epilogue (its group is the active group of tile Q - 1)
  if (((Q - 1) & 1) == grp) {
#pragma unroll
    for (int j = 0; j < 8; ++j) epi_j(p, acc, j, ep_m0, ep_n0, wm, wn, ry);
  }
}


// Variant 2: the inactive group issues ALL operand DMA (an LDS-DMA piece costs its issuing wave ~60 cycles:
// the MFMA wave issues only ds_reads and MFMAs).  FL bit 0: no DMA waits (timing only), bit 1: no epilogue.
template <int R, int FL>
__global__ __launch_bounds__(512) void pp2_gemm(Params p, int tiles_m, int tiles_n) {
  static_assert(R == 5, "wait ladders written for R = 5");
  constexpr int E0 = 1, ES = 2;  // epilogue chunk j at inactive iteration E0 + j * ES
  __shared__ __attribute__((aligned(1024))) h16 smem[R * STAGE];
  const int ntiles = tiles_m * tiles_n;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int grp = wave >> 2, gw = wave & 3;
  const int wm = gw & 1, wn = gw >> 1;
  const int Q = ntiles > (int)blockIdx.x ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int nk = p.K / BK;
  const int total = Q * nk;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)((long)p.M * p.K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)((long)p.N * p.K * 2), 0x00020000);
  auto foff_of = [](int lane) {
    const int frow = lane & 15, fchunk = lane >> 4;
    return frow * BK + ((fchunk ^ (-(frow >> 2) & 3)) << 3);
  };
  unsigned voff[PPW];
  auto set_tile_dma = [&](int q) {
    const int vb = (int)blockIdx.x + q * (int)gridDim.x;
    int tm, tn;
    tile_coords(vb, ntiles, tiles_m, tiles_n, tm, tn);
    const int lane = vlane();
    const int dlr = lane >> 2;
    const int dlc = ((lane & 3) ^ (-(dlr >> 2) & 3)) * 8;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pi = gw + 4 * i;
      if (i < 4) {
        const int m = tm * BM + pi * 16 + dlr;
        voff[i] = m < p.M ? (unsigned)(((long)m * p.K + dlc) * 2) : 0x80000000u;
      } else {
        const int n = tn * BN + (pi - 16) * 16 + dlr;
        voff[i] = n < p.N ? (unsigned)(((long)n * p.K + dlc) * 2) : 0x80000000u;
      }
    }
  };
  auto issue = [&](int s) {
    const int kk = s % nk;
    h16* sb = smem + (s % R) * STAGE;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pi = gw + 4 * i;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 4 ? xrs : wrs, (VDA_LDS void*)(sb + pi * 512), 16, (int)voff[i],
                                               kk * BK * 2, 0, 0);
    }
  };
  h8 xf[8], wf[4];
  auto read_x = [&](int s, int j, int fo) {
    xf[j] = *reinterpret_cast<const h8*>(smem + (s % R) * STAGE + fo + (wm * 128 + j * 16) * BK);
  };
  auto read_w = [&](int s, int fo) {
    const h16* sb = smem + (s % R) * STAGE + fo;
#pragma unroll
    for (int i = 0; i < 4; ++i) wf[i] = *reinterpret_cast<const h8*>(sb + (BM + wn * 64 + i * 16) * BK);
  };
  auto read_frags = [&](int s) {
    const int fo = foff_of(vlane());
    read_w(s, fo);
#pragma unroll
    for (int j = 0; j < 8; ++j) read_x(s, j, fo);
  };
  // stores issued after the DMA of stage t (iteration t - R + 1 of the issuing group) and before the
  // wait for it: chunks in iterations (a, b] of the same tile
  auto chunks_in = [&](int a, int b) {  // # of E0 + j * ES in [a, b], j < 8
    int c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) c += (E0 + j * ES >= a && E0 + j * ES <= b) ? 1 : 0;
    return c;
  };
  auto wait_dyn = [&](int c) {  // wait until at most 6(R-3) + 2c ops are outstanding
    if (FL & 1) return;
    switch (c) {
      case 0: wait_vm<(R - 3) * PPW>(); break;
      case 1: wait_vm<(R - 3) * PPW + 2>(); break;
      case 2: wait_vm<(R - 3) * PPW + 4>(); break;
      default: wait_vm<(R - 3) * PPW + 6>(); break;
    }
  };
  f4 acc[4][8];
  if (Q == 0) return;
  // prologue: group 1 (inactive during tile 0) issues stages 0 .. R-2
  if (grp == 1) {
    set_tile_dma(0);
    for (int s = 0; s < R - 1 && s < total; ++s) {
      if (s == nk) set_tile_dma(1);
      issue(s);
    }
    if (!(FL & 1)) wait_vm<(R - 2) * PPW>();
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 0) read_frags(0);
  int ep_m0 = 0, ep_n0 = 0;
  __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void*)p.y, (short)0, 0, 0x00020000);
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using BT = std::integral_constant<bool, true>;
  using BF = std::integral_constant<bool, false>;

  for (int q = 0; q < Q; ++q) {
    const bool active = (q & 1) == grp;
    if (active) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
      const int fo = foff_of(vlane());
      auto kstep = [&](int kk, auto rc) {
        constexpr bool rd = decltype(rc)::value;
        const int s = q * nk + kk;
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][j] = mfma16(wf[i], xf[j], acc[i][j]);
          if (rd) read_x(s + 1, j, fo);
        }
        if (rd) read_w(s + 1, fo);
      };
      // stages q*nk + 1 .. q*nk + R - 2 were issued by this group during tile q - 1 (after its stores)
      if (q >= 1) {
        if (!(FL & 1)) wait_vm<2 * PPW>();
        kstep(0, BT{});
        if (!(FL & 1)) wait_vm<1 * PPW>();
        kstep(1, BT{});
        if (!(FL & 1)) wait_vm<0>();
        kstep(2, BT{});
      } else {
        kstep(0, BT{}); kstep(1, BT{}); kstep(2, BT{});
      }
      for (int kk = 3; kk < nk - 1; ++kk) kstep(kk, BT{});
      kstep(nk - 1, BF{});
      const int vb = (int)blockIdx.x + q * (int)gridDim.x;
      int tm, tn;
      tile_coords(vb, ntiles, tiles_m, tiles_n, tm, tn);
      ep_m0 = tm * BM;
      ep_n0 = tn * BN;
      const long mrows = p.M - ep_m0;
      ry = __builtin_amdgcn_make_buffer_rsrc((void*)(p.y + (long)ep_m0 * p.N), (short)0,
                                             (int)(mrows * p.N * 2 < 0x7fffffffL ? mrows * p.N * 2 : 0x7fffffffL), 0x00020000);
    } else {
      // inactive: DMA of stage s + R - 1 each iteration, the previous tile's epilogue in 8 chunks
      if (q > 0) set_tile_dma(q);
      const bool epi = q >= 1 && !(FL & 2);
      for (int kk = 0; kk < nk; ++kk) {
        const int s = q * nk + kk;
        // my pieces of stage s + 1 (issued at iteration kk + 2 - R of this tile; at q == 0 also the prologue)
        if (kk >= R - 2 || q == 0) wait_dyn(epi ? chunks_in(kk + 2 - R, kk - 1) : 0);
        __builtin_amdgcn_s_barrier();
        if (s + R - 1 < total) {
          if (kk + R - 1 == nk) set_tile_dma(q + 1);
          issue(s + R - 1);
        }
        if (epi && kk >= E0 && kk < E0 + 8 * ES && ((kk - E0) % ES) == 0) {
          const int jj = (kk - E0) / ES;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j == jj) epi_j(p, acc, j, ep_m0, ep_n0, wm, wn, ry);
        }
      }
      if (q + 1 < Q) read_frags((q + 1) * nk);
    }
  }
  if (((Q - 1) & 1) == grp && (!(FL & 2) || p.M < 0)) {  // FL 2: keep the MFMAs alive
#pragma unroll
    for (int j = 0; j < 8; ++j) epi_j(p, acc, j, ep_m0, ep_n0, wm, wn, ry);
  }
}

__global__ void ref_gemm(const h16* x, const h16* w, float* y, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)x[(long)m * K + k] * (float)w[(long)n * K + k];
  y[(long)m * N + n] = s;
}
__global__ void init_rand(h16* a, long n, unsigned seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned v = (unsigned)i * 2654435761u ^ seed;
    v ^= v >> 13; v *= 0x5bd1e995u; v ^= v >> 15;
    a[i] = (h16)(((float)(v & 0xffff) / 65535.f * 2.f - 1.f) * scale);
  }
}
}  // namespace pp

int main(int argc, char** argv) {
  using namespace pp;
  const int M = 43840;
  struct Shape { const char* name; int N, K; } shapes[] = {{"qkv", 3072, 1024}, {"proj", 1024, 1024}, {"fc1", 4096, 1024}, {"fc2", 1024, 4096}};
  typedef void (*KFn)(Params, int, int);
  struct Var { const char* name; KFn fn; bool check; } vars[] = {
      {"pp1", pp_gemm<5>, true},
      {"pp2", pp2_gemm<5, 0>, true},
      {"pp2-nowait", pp2_gemm<5, 1>, false},
      {"pp2-noepi", pp2_gemm<5, 2>, false},
  };
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (auto& sh : shapes) {
    const int N = sh.N, K = sh.K;
    h16 *x, *w, *y;
    float* yr;
    CK(hipMalloc(&x, (size_t)M * K * 2)); CK(hipMalloc(&w, (size_t)N * K * 2)); CK(hipMalloc(&y, (size_t)M * N * 2));
    CK(hipMalloc(&yr, (size_t)M * N * 4));
    init_rand<<<2048, 256>>>(x, (long)M * K, 1, 1.f);
    init_rand<<<2048, 256>>>(w, (long)N * K, 2, 1.f / sqrtf((float)K));
    Params prm{x, w, y, nullptr, M, N, K};
    const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
    const int grid = std::min(cus, tiles_m * tiles_n);
    const int Mc = 1024;
    std::vector<h16> hy((size_t)Mc * N);
    std::vector<float> hr0((size_t)Mc * N), hr1((size_t)Mc * N);
    ref_gemm<<<dim3((N + 255) / 256, Mc), 256>>>(x, w, yr, Mc, N, K);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hr0.data(), yr, hr0.size() * 4, hipMemcpyDeviceToHost));
    ref_gemm<<<dim3((N + 255) / 256, Mc), 256>>>(x + (long)(M - Mc) * K, w, yr, Mc, N, K);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hr1.data(), yr, hr1.size() * 4, hipMemcpyDeviceToHost));
    for (auto& v : vars) {
      double rel = -1;
      if (v.check) {
        CK(hipMemset(y, 0, (size_t)M * N * 2));
        v.fn<<<grid, 512>>>(prm, tiles_m, tiles_n);
        CK(hipDeviceSynchronize());
        double se = 0, sr = 0;
        CK(hipMemcpy(hy.data(), y, hy.size() * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < hy.size(); ++i) { se += fabs((double)(float)hy[i] - hr0[i]); sr += fabs(hr0[i]); }
        CK(hipMemcpy(hy.data(), y + (long)(M - Mc) * N, hy.size() * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < hy.size(); ++i) { se += fabs((double)(float)hy[i] - hr1[i]); sr += fabs(hr1[i]); }
        rel = se / sr;
      }
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
      std::vector<float> ts;
      for (int it = 0; it < 12; ++it) {
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) v.fn<<<grid, 512>>>(prm, tiles_m, tiles_n);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms * 1000.f / 5);
      }
      std::sort(ts.begin(), ts.end());
      const double fl = 2.0 * M * N * K;
      printf("%-5s %-11s N=%d K=%d tiles %d (%.2f rounds): med %.1f us min %.1f us  %.0f TF  rel-L1 %.2e\n", sh.name, v.name,
             N, K, tiles_m * tiles_n, (double)tiles_m * tiles_n / grid, ts[ts.size() / 2], ts[0],
             fl / ts[ts.size() / 2] * 1e-6, rel);
      fflush(stdout);
      CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
    }
    CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(y)); CK(hipFree(yr));
  }
  return 0;
}
