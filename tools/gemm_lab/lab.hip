// GEMM structure lab (tuning tool, not product code): Y[M, N] = X[M, K] W[N, K]^T + bias, fp16 in / out,
// fp32 accumulation, on structures that the product's phased kernel (vda_gemm.hip) does not use.
//
// w4: 256 x 256 tile, 4 waves (ONE per SIMD, 512-register budget), wave tile 128 x 128 (64 accumulators
// of 16x16 in AGPRs), K steps of 32 through a 4-stage LDS ring filled by buffer_load ... lds, one barrier
// per K step, the next step's fragments read from LDS under this step's MFMAs (register double buffer).
// Per 32-deep K step and CU: 32 KiB staged, 128 KiB of fragment reads (the 8-wave 128 x 64 layout reads
// 192-224 KiB per 64-deep step, i.e. 96-112 KiB per 32), one barrier instead of four.
#include "../../video-depth-anything_amd/csrc/vda_common.h"
#include <utility>

namespace {

constexpr int BK = 32, NS = 4;
constexpr int STAGE = 512 * BK;  // halves per stage: X 256 rows + W 256 rows of 32 halves (32 KiB)

struct LabParams {
  const h16* x;
  const h16* w;
  h16* y;
  const float* bias;
  int M, N, K;
};

// 16-B chunk swizzle of a [rows][32 halves] image: the 16x16x32 fragment reads (row = lane & 15,
// chunk = lane >> 4) are conflict-free in every ds_read_b128 lane group
__device__ __forceinline__ int swz(int row) { return (-(row >> 2)) & 3; }

__device__ __forceinline__ void tile_coords(int bid, int nwg, int tiles_m, int tiles_n, int& tm, int& tn) {
  constexpr int GROUP_M = 8;
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

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7F << 4) /* lgkm, exp: no wait */);
}
__device__ __forceinline__ void wait_vm_dyn(int n) {  // n in {0, 8, 16, 24}
  if (n >= 24) wait_vm<24>();
  else if (n >= 16) wait_vm<16>();
  else if (n >= 8) wait_vm<8>();
  else wait_vm<0>();
}

__device__ __forceinline__ void perm16_swap(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}

// MFMA through asm with the accumulator pinned to AGPRs in place (no accumulator copies by the
// register allocator); the hazard recognizer does not see inside: the epilogue pads before it reads
__device__ __forceinline__ void mfma_a(f4& c, h8 a, h8 b) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ h8 lds_frag(const h16* smem, unsigned byte_off) {
  return *reinterpret_cast<const h8*>(reinterpret_cast<const char*>(smem) + byte_off);
}

template <int VAR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void w4_kernel(LabParams p, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(1024))) h16 smem[NS * STAGE];
  int lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int ntiles = tiles_m * tiles_n;
  const int nk = p.K / BK;
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)((long)p.M * p.K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)((long)p.N * p.K * 2), 0x00020000);
  // DMA piece q (0..15) of an operand = rows 16q .. 16q + 15: lane -> row 16q + (lane >> 2), LDS slot
  // lane & 3, source chunk slot ^ swz(row); wave w issues pieces 4w .. 4w + 3 of X and of W
  const int prow = lane >> 2;
  const int pch = (lane & 3) ^ swz(prow);
  // fragment read: row 16 blk + (lane & 15), chunk lane >> 4 -> byte offset (lane constant + immediates)
  const int frow = lane & 15, fch = lane >> 4;
  const unsigned fofs = (unsigned)(frow * BK + ((fch ^ swz(frow)) << 3)) * 2u;
  const unsigned xfo = fofs + (unsigned)(wm * 128 * BK * 2);
  const unsigned wfo = fofs + (unsigned)((256 + wn * 128) * BK * 2);
  const unsigned sbase = (unsigned)(uintptr_t)(VDA_LDS h16*)smem;

  f4 acc[8][8];
  h8 fx[2][8], fw[2][8];
  int vb = blockIdx.x;
  unsigned xo[4], wo[4];
  auto offsets = [&](int vb_) {
    int tm, tn;
    tile_coords(vb_, ntiles, tiles_m, tiles_n, tm, tn);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (wave * 4 + i) * 16 + prow;
      const int m = tm * 256 + r, n = tn * 256 + r;
      xo[i] = m < p.M ? (unsigned)(((long)m * p.K + pch * 8) * 2) : 0x80000000u;
      wo[i] = n < p.N ? (unsigned)(((long)n * p.K + pch * 8) * 2) : 0x80000000u;
    }
  };
  auto dma = [&](int t) {
    h16* sb = smem + (t & 3) * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (VDA_LDS void*)(sb + (wave * 4 + i) * 512), 16, (int)xo[i], t * BK * 2, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (VDA_LDS void*)(sb + 256 * BK + (wave * 4 + i) * 512), 16, (int)wo[i], t * BK * 2, 0, 0);
  };
  auto read_frags = [&](int t, h8 (&gx)[8], h8 (&gw)[8]) {
    const h16* sb = smem + (t & 3) * STAGE;
#pragma unroll
    for (int j = 0; j < 8; ++j) gx[j] = lds_frag(sb, xfo + j * 16 * BK * 2);
#pragma unroll
    for (int i = 0; i < 8; ++i) gw[i] = lds_frag(sb, wfo + i * 16 * BK * 2);
  };
  (void)sbase;

  if (vb < ntiles) {
    offsets(vb);
    for (int s = 0; s < NS; ++s) dma(s);
  }
  for (; vb < ntiles; vb += gridDim.x) {
    int tm, tn;
    tile_coords(vb, ntiles, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    // prologue DMA(0 .. 3) was issued (first tile above, later tiles by the previous tile's last step);
    // the previous epilogue's 32 stores are younger than all of it
    if (vb == (int)blockIdx.x) wait_vm<24>();
    else wait_vm<56>();
    __builtin_amdgcn_s_barrier();
    read_frags(0, fx[0], fw[0]);
    const int vb_next = vb + (int)gridDim.x;

    // one K step: the fragments of step t are in register set S; DMA(t + 1) must have landed (WAIT =
    // the vector-memory operations younger than it), then the barrier publishes it and frees stage
    // t & 3 (its reads, for step t, were waited for before the barrier by every wave)
    auto step = [&](int t, auto setc, auto waitc, auto dmac, auto readc) {
      constexpr int S = decltype(setc)::value;
      constexpr int WAIT = decltype(waitc)::value;   // -1: no vmcnt wait
      constexpr int DMA = decltype(dmac)::value;     // 0 none, 1 DMA(t + 4), 2 the next tile's prologue
      constexpr bool READ = decltype(readc)::value;
      if constexpr (WAIT >= 0) wait_vm<WAIT>();
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      if constexpr (DMA == 1) dma(t + 4);
      if constexpr (DMA == 2) {
        if (vb_next < ntiles) {
          offsets(vb_next);
#pragma unroll
          for (int s = 0; s < NS; ++s) dma(s);
        }
      }
      if constexpr (READ) {
        const h16* sb = smem + ((t + 1) & 3) * STAGE;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if constexpr (VAR & 2) mfma_a(acc[i][j], fw[S][i], fx[S][j]);
            else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[S][i], fx[S][j], acc[i][j], 0, 0, 0);
            if (j == 3) fx[S ^ 1][i] = lds_frag(sb, xfo + i * 16 * BK * 2);
            if (j == 7) fw[S ^ 1][i] = lds_frag(sb, wfo + i * 16 * BK * 2);
          }
          if constexpr (!(VAR & 1)) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if constexpr (VAR & 2) mfma_a(acc[i][j], fw[S][i], fx[S][j]);
            else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[S][i], fx[S][j], acc[i][j], 0, 0, 0);
          }
        if constexpr (VAR & 2) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7");
      }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using W16 = std::integral_constant<int, 16>;
    using W8 = std::integral_constant<int, 8>;
    using W0 = std::integral_constant<int, 0>;
    using WN = std::integral_constant<int, -1>;
    using RT = std::integral_constant<bool, true>;
    using RF = std::integral_constant<bool, false>;
    // steady state (nk even, >= 6: the host checks): DMA(t + 4) issued, DMA(t + 2), (t + 3) younger than t + 1
    for (int t = 0; t < nk - 4; t += 2) {
      step(t, I0{}, W16{}, I1{}, RT{});
      step(t + 1, I1{}, W16{}, I1{}, RT{});
    }
    step(nk - 4, I0{}, W16{}, I0{}, RT{});
    step(nk - 3, I1{}, W8{}, I0{}, RT{});
    step(nk - 2, I0{}, W0{}, I0{}, RT{});
    step(nk - 1, I1{}, WN{}, I2{}, RF{});

    // epilogue: + bias, fp16; v_permlane16_swap pairs blocks (2pp, 2pp + 1) so a lane holds 8 consecutive
    // channels, a DPP row_ror:8 exchange gives whole 128-B lines per 16-B store
    const int mcol = lane & 15, g = lane >> 4;
    const bool lo8 = (mcol & 8) == 0;
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.y, (short)0, (int)((long)p.M * p.N * 2 < 0x7fffffffL ? (long)p.M * p.N * 2 : 0x7fffffffL), 0x00020000);
    f4 bv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int n = n0 + wn * 128 + i * 16 + g * 4;
      bv[i] = n < p.N ? *reinterpret_cast<const f4*>(p.bias + n) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) {  // channel halves 0..63, 64..127 of the wave's 128
        u32x4 o[2];
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int ia = hl * 4 + 2 * pp;
          float a[4], c[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            a[r] = acc[ia][j][r] + bv[ia][r];
            c[r] = acc[ia + 1][j][r] + bv[ia + 1][r];
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
        const int col = n0 + wn * 128 + hl * 64 + 32 * (lo8 ? 0 : 1) + 16 * (g & 1) + 8 * (g >> 1);
        const int rowA = m0 + wm * 128 + j * 16 + (mcol & 7);
        const bool okc = col < p.N;
        const unsigned oA = okc && rowA < p.M ? (unsigned)(((long)rowA * p.N + col) * 2) : 0x80000000u;
        const unsigned oB = okc && rowA + 8 < p.M ? (unsigned)(((long)(rowA + 8) * p.N + col) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(A, ry, oA, 0, 2);
        __builtin_amdgcn_raw_buffer_store_b128(B, ry, oB, 0, 2);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
}


// ---- w4b: w4 with every DMA and MFMA placed by hand (asm), reads pinned between them, bias via LDS ----
typedef int i4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i4v rsrc4(const void* p, long bytes) {
  const unsigned long a = (unsigned long)p;
  return i4v{(int)(unsigned)a, (int)(unsigned)(a >> 32), (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL), 0x00020000};
}
__device__ __forceinline__ void dma16(i4v rs, unsigned voff, int soff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rs), "s"(soff), "s"(lds)
               : "memory", "m0");
}
__device__ __forceinline__ void mfma_m(f4& c, h8 a, h8 b) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b) : "memory");
}
// first K step of a tile: C = 0 (no accumulator initialisation, no VALU-write -> MFMA-read hazard that
// the hazard recognizer would not see through the asm)
__device__ __forceinline__ void mfma_z(f4& c, h8 a, h8 b) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b) : "memory");
}

constexpr int BIAS_OFS = NS * STAGE;  // halves: two 1-KiB bias slots after the stages

// RD: reads spread every RD MFMAs from the start of the step; DS: one DMA piece every DS MFMAs from DOF
template <int RD, int DS, int DOF, int FL = 0>  // FL timing-only probes: 1 no loop DMA, 2 no MFMA, 4 no reads
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void w4b_kernel(LabParams p, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(1024))) h16 smem[NS * STAGE + 1024];
  int lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int ntiles = tiles_m * tiles_n;
  const int nk = p.K / BK;
  const i4v xrs = rsrc4(p.x, (long)p.M * p.K * 2), wrs = rsrc4(p.w, (long)p.N * p.K * 2);
  const i4v brs = rsrc4(p.bias, (long)p.N * 4);
  const int prow = lane >> 2;
  const int pch = (lane & 3) ^ swz(prow);
  const int frow = lane & 15, fch = lane >> 4;
  const unsigned fofs = (unsigned)(frow * BK + ((fch ^ swz(frow)) << 3)) * 2u;
  const unsigned xfo = fofs + (unsigned)(wm * 128 * BK * 2);
  const unsigned wfo = fofs + (unsigned)((256 + wn * 128) * BK * 2);
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(VDA_LDS h16*)smem);

  f4 acc[8][8];
  h8 fx[2][8], fw[2][8];
  int vb = blockIdx.x;
  unsigned xo[4], wo[4], bo = 0;
  int cnt = 0;  // tiles this block has started (bias slot parity)
  auto offsets = [&](int vb_) {
    int tm, tn;
    tile_coords(vb_, ntiles, tiles_m, tiles_n, tm, tn);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (wave * 4 + i) * 16 + prow;
      const int m = tm * 256 + r, n = tn * 256 + r;
      xo[i] = m < p.M ? (unsigned)(((long)m * p.K + pch * 8) * 2) : 0x80000000u;
      wo[i] = n < p.N ? (unsigned)(((long)n * p.K + pch * 8) * 2) : 0x80000000u;
    }
    const int nb = tn * 256 + lane * 4;
    bo = nb < p.N ? (unsigned)(nb * 4) : 0x80000000u;
  };
  auto piece = [&](int t, int q) {  // DMA piece q (0..7) of step t: X pieces 0-3, W pieces 4-7
    const unsigned sb = lds0 + (unsigned)((t & 3) * STAGE * 2);
    if (q < 4) dma16(xrs, xo[q], t * BK * 2, sb + (unsigned)((wave * 4 + q) * 1024));
    else dma16(wrs, wo[q - 4], t * BK * 2, sb + (unsigned)((256 * BK + (wave * 4 + q - 4) * 512) * 2));
  };
  auto prologue = [&](int slot) {  // DMA(0 .. 3) (+ the tile's bias row by wave 0) for the tile offsets() set up
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int q = 0; q < 8; ++q) piece(s, q);
    if (wave == 0) dma16(brs, bo, 0, lds0 + (unsigned)((BIAS_OFS + slot * 512) * 2));
  };
  if (vb < ntiles) {
    offsets(vb);
    prologue(0);
  }
  for (; vb < ntiles; vb += gridDim.x, ++cnt) {
    int tm, tn;
    tile_coords(vb, ntiles, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    // DMA(0) landed: younger are DMA(1 .. 3) (24, + wave 0's bias piece) and the previous epilogue's 32 stores
    if (vb == (int)blockIdx.x) {
      if (wave == 0) wait_vm<25>(); else wait_vm<24>();
    } else {
      if (wave == 0) wait_vm<57>(); else wait_vm<56>();
    }
    __builtin_amdgcn_s_barrier();
    {
      const h16* sb = smem;
#pragma unroll
      for (int j = 0; j < 8; ++j) fx[0][j] = lds_frag(sb, xfo + j * 16 * BK * 2);
#pragma unroll
      for (int i = 0; i < 8; ++i) fw[0][i] = lds_frag(sb, wfo + i * 16 * BK * 2);
    }
    const int vb_next = vb + (int)gridDim.x;

    auto step = [&](int t, auto setc, auto waitc, auto dmac, auto readc, auto zc) {
      constexpr bool Z = decltype(zc)::value;
      constexpr int S = decltype(setc)::value;
      constexpr int WAIT = decltype(waitc)::value;
      constexpr int DMA = decltype(dmac)::value;  // 0 none, 1 DMA(t + 4), 2 the next tile's prologue
      constexpr bool READ = decltype(readc)::value;
      if constexpr (WAIT >= 0) wait_vm<WAIT>();
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
      if constexpr (DMA == 2) {
        if (vb_next < ntiles) {
          offsets(vb_next);
          prologue((cnt + 1) & 1);
        }
      }
      const h16* sb = smem + ((t + 1) & 3) * STAGE;
#pragma unroll
      for (int mi = 0; mi < 64; ++mi) {
        const int i = mi >> 3, j = mi & 7;
        if constexpr (FL & 2) {
          if (mi == 0) mfma_m(acc[i][j], fw[S][i], fx[S][j]);
        } else if constexpr (Z) mfma_z(acc[i][j], fw[S][i], fx[S][j]);
        else mfma_m(acc[i][j], fw[S][i], fx[S][j]);
        if constexpr (READ && !(FL & 4)) {
          if (mi % RD == 0 && mi / RD < 16) {
            const int r = mi / RD;
            if (r < 8) fx[S ^ 1][r] = lds_frag(sb, xfo + r * 16 * BK * 2);
            else fw[S ^ 1][r - 8] = lds_frag(sb, wfo + (r - 8) * 16 * BK * 2);
          }
        }
        if constexpr (DMA == 1 && !(FL & 1)) {
          if (mi >= DOF && mi % DS == DOF % DS && (mi - DOF) / DS < 8) piece(t + 4, (mi - DOF) / DS);
        }
      }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using W16 = std::integral_constant<int, 16>;
    using W8 = std::integral_constant<int, 8>;
    using W0 = std::integral_constant<int, 0>;
    using WN = std::integral_constant<int, -1>;
    using RT = std::integral_constant<bool, true>;
    using RF = std::integral_constant<bool, false>;
    step(0, I0{}, W16{}, I1{}, RT{}, std::true_type{});
    step(1, I1{}, W16{}, I1{}, RT{}, std::false_type{});
    for (int t = 2; t < nk - 4; t += 2) {
      step(t, I0{}, W16{}, I1{}, RT{}, std::false_type{});
      step(t + 1, I1{}, W16{}, I1{}, RT{}, std::false_type{});
    }
    step(nk - 4, I0{}, W16{}, I0{}, RT{}, std::false_type{});
    step(nk - 3, I1{}, W8{}, I0{}, RT{}, std::false_type{});
    step(nk - 2, I0{}, W0{}, I0{}, RT{}, std::false_type{});
    step(nk - 1, I1{}, WN{}, I2{}, RF{}, std::false_type{});
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

    const int mcol = lane & 15, g = lane >> 4;
    const bool lo8 = (mcol & 8) == 0;
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.y, (short)0, (int)((long)p.M * p.N * 2 < 0x7fffffffL ? (long)p.M * p.N * 2 : 0x7fffffffL), 0x00020000);
    f4 bv[8];
    {
      const float* bl = reinterpret_cast<const float*>(smem + BIAS_OFS + (cnt & 1) * 512);
#pragma unroll
      for (int i = 0; i < 8; ++i) bv[i] = *reinterpret_cast<const f4*>(bl + wn * 128 + i * 16 + g * 4);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) {
        u32x4 o[2];
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int ia = hl * 4 + 2 * pp;
          float a[4], c[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            a[r] = acc[ia][j][r] + bv[ia][r];
            c[r] = acc[ia + 1][j][r] + bv[ia + 1][r];
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
        const int col = n0 + wn * 128 + hl * 64 + 32 * (lo8 ? 0 : 1) + 16 * (g & 1) + 8 * (g >> 1);
        const int rowA = m0 + wm * 128 + j * 16 + (mcol & 7);
        const bool okc = col < p.N;
        const unsigned oA = okc && rowA < p.M ? (unsigned)(((long)rowA * p.N + col) * 2) : 0x80000000u;
        const unsigned oB = okc && rowA + 8 < p.M ? (unsigned)(((long)(rowA + 8) * p.N + col) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(A, ry, oA, 0, 2);
        __builtin_amdgcn_raw_buffer_store_b128(B, ry, oB, 0, 2);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
}

template <int RD, int DS, int DOF, int FL, int NST>  // w4b with NST stages in the ring (FL 8: no bias)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void w4c_kernel(LabParams p, int tiles_m, int tiles_n) {
  constexpr bool LB = NST * STAGE + 1024 <= 81920 && !(FL & 8);  // bias row staged in LDS
  __shared__ __attribute__((aligned(1024))) h16 smem[NST * STAGE + (LB ? 1024 : 0)];
  constexpr int BOFS = NST * STAGE;
  int lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int ntiles = tiles_m * tiles_n;
  const int nk = p.K / BK;
  const i4v xrs = rsrc4(p.x, (long)p.M * p.K * 2), wrs = rsrc4(p.w, (long)p.N * p.K * 2);
  const i4v brs = rsrc4(p.bias, (long)p.N * 4);
  const int prow = lane >> 2;
  const int pch = (lane & 3) ^ swz(prow);
  const int frow = lane & 15, fch = lane >> 4;
  const unsigned fofs = (unsigned)(frow * BK + ((fch ^ swz(frow)) << 3)) * 2u;
  const unsigned xfo = fofs + (unsigned)(wm * 128 * BK * 2);
  const unsigned wfo = fofs + (unsigned)((256 + wn * 128) * BK * 2);
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(VDA_LDS h16*)smem);

  f4 acc[8][8];
  h8 fx[2][8], fw[2][8];
  int vb = blockIdx.x;
  unsigned xo[4], wo[4], bo = 0;
  int cnt = 0;  // tiles this block has started (bias slot parity)
  auto offsets = [&](int vb_) {
    int tm, tn;
    tile_coords(vb_, ntiles, tiles_m, tiles_n, tm, tn);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (wave * 4 + i) * 16 + prow;
      const int m = tm * 256 + r, n = tn * 256 + r;
      xo[i] = m < p.M ? (unsigned)(((long)m * p.K + pch * 8) * 2) : 0x80000000u;
      wo[i] = n < p.N ? (unsigned)(((long)n * p.K + pch * 8) * 2) : 0x80000000u;
    }
    const int nb = tn * 256 + lane * 4;
    bo = nb < p.N ? (unsigned)(nb * 4) : 0x80000000u;
  };
  auto piece = [&](int t, int q) {  // DMA piece q (0..7) of step t: X pieces 0-3, W pieces 4-7
    const unsigned sb = lds0 + (unsigned)((t % NST) * STAGE * 2);
    if (q < 4) dma16(xrs, xo[q], t * BK * 2, sb + (unsigned)((wave * 4 + q) * 1024));
    else dma16(wrs, wo[q - 4], t * BK * 2, sb + (unsigned)((256 * BK + (wave * 4 + q - 4) * 512) * 2));
  };
  auto prologue = [&](int slot) {  // DMA(0 .. 3) (+ the tile's bias row by wave 0) for the tile offsets() set up
#pragma unroll
    for (int s = 0; s < NST; ++s)
#pragma unroll
      for (int q = 0; q < 8; ++q) piece(s, q);
    if (LB && wave == 0) dma16(brs, bo, 0, lds0 + (unsigned)((BOFS + slot * 512) * 2));
  };
  if (vb < ntiles) {
    offsets(vb);
    prologue(0);
  }
  for (; vb < ntiles; vb += gridDim.x, ++cnt) {
    int tm, tn;
    tile_coords(vb, ntiles, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    // DMA(0) landed: younger are DMA(1 .. 3) (24, + wave 0's bias piece) and the previous epilogue's 32 stores
    constexpr int YP = (NST - 1) * 8;  // prologue pieces younger than DMA(0)
    if (vb == (int)blockIdx.x) {
      if (LB && wave == 0) wait_vm<YP + 1>(); else wait_vm<YP>();
    } else {
      if (LB && wave == 0) wait_vm<(YP + 33 < 63 ? YP + 33 : 63)>(); else wait_vm<(YP + 32 < 63 ? YP + 32 : 63)>();
    }
    __builtin_amdgcn_s_barrier();
    {
      const h16* sb = smem;
#pragma unroll
      for (int j = 0; j < 8; ++j) fx[0][j] = lds_frag(sb, xfo + j * 16 * BK * 2);
#pragma unroll
      for (int i = 0; i < 8; ++i) fw[0][i] = lds_frag(sb, wfo + i * 16 * BK * 2);
    }
    const int vb_next = vb + (int)gridDim.x;

    auto step = [&](int t, auto setc, auto waitc, auto dmac, auto readc, auto zc) {
      constexpr bool Z = decltype(zc)::value;
      constexpr int S = decltype(setc)::value;
      constexpr int WAIT = decltype(waitc)::value;
      constexpr int DMA = decltype(dmac)::value;  // 0 none, 1 DMA(t + NST), 2 the next tile's prologue
      constexpr bool READ = decltype(readc)::value;
      if constexpr (WAIT >= 0) wait_vm<WAIT>();
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
      if constexpr (DMA == 2) {
        if (vb_next < ntiles) {
          offsets(vb_next);
          prologue((cnt + 1) & 1);
        }
      }
      const h16* sb = smem + ((t + 1) % NST) * STAGE;
#pragma unroll
      for (int mi = 0; mi < 64; ++mi) {
        const int i = mi >> 3, j = mi & 7;
        if constexpr (FL & 2) {
          if (mi == 0) mfma_m(acc[i][j], fw[S][i], fx[S][j]);
        } else if constexpr (Z) mfma_z(acc[i][j], fw[S][i], fx[S][j]);
        else mfma_m(acc[i][j], fw[S][i], fx[S][j]);
        if constexpr (READ && !(FL & 4)) {
          if (mi % RD == 0 && mi / RD < 16) {
            const int r = mi / RD;
            if (r < 8) fx[S ^ 1][r] = lds_frag(sb, xfo + r * 16 * BK * 2);
            else fw[S ^ 1][r - 8] = lds_frag(sb, wfo + (r - 8) * 16 * BK * 2);
          }
        }
        if constexpr (DMA == 1 && !(FL & 1)) {
          if (mi >= DOF && mi % DS == DOF % DS && (mi - DOF) / DS < 8) piece(t + NST, (mi - DOF) / DS);
        }
      }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using WS = std::integral_constant<int, 8 * (NST - 2)>;
    using RT = std::integral_constant<bool, true>;
    using FT = std::false_type;
    // steady state: t = 0 .. nk - NST - 1 (DMA(t + NST) issued, DMA(t + 2 .. t + NST - 1) younger than t + 1)
    step(0, I0{}, WS{}, I1{}, RT{}, std::true_type{});
    int t = 1;
    if constexpr (NST % 2 == 0) {  // nk even: nk - NST has NST's parity; step 1 alone, then pairs from 2
      step(1, I1{}, WS{}, I1{}, RT{}, FT{});
      t = 2;
      for (; t < nk - NST; t += 2) {
        step(t, I0{}, WS{}, I1{}, RT{}, FT{});
        step(t + 1, I1{}, WS{}, I1{}, RT{}, FT{});
      }
    } else {
      for (; t < nk - NST; t += 2) {
        step(t, I1{}, WS{}, I1{}, RT{}, FT{});
        step(t + 1, I0{}, WS{}, I1{}, RT{}, FT{});
      }
    }
    // the last NST steps (nk even: step nk - NST + u has parity (NST + u) & 1)
    [&]<int... U>(std::integer_sequence<int, U...>) {
      (([&] {
         constexpr int u = U;
         using SU = std::integral_constant<int, (NST + u) & 1>;
         if constexpr (u == NST - 1) {
           step(nk - 1, SU{}, std::integral_constant<int, -1>{}, I2{}, std::false_type{}, FT{});
         } else {
           step(nk - NST + u, SU{}, std::integral_constant<int, 8 * (NST - u - 2 > 0 ? NST - u - 2 : 0)>{}, I0{}, RT{}, FT{});
         }
       }()), ...);
    }(std::make_integer_sequence<int, NST>{});
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

    const int mcol = lane & 15, g = lane >> 4;
    const bool lo8 = (mcol & 8) == 0;
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.y, (short)0, (int)((long)p.M * p.N * 2 < 0x7fffffffL ? (long)p.M * p.N * 2 : 0x7fffffffL), 0x00020000);
    f4 bv[8];
    {
      const float* bl = reinterpret_cast<const float*>(smem + BOFS + (cnt & 1) * 512);
#pragma unroll
      for (int i = 0; i < 8; ++i) bv[i] = LB ? *reinterpret_cast<const f4*>(bl + wn * 128 + i * 16 + g * 4) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) {
        u32x4 o[2];
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int ia = hl * 4 + 2 * pp;
          float a[4], c[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            a[r] = acc[ia][j][r] + bv[ia][r];
            c[r] = acc[ia + 1][j][r] + bv[ia + 1][r];
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
        const int col = n0 + wn * 128 + hl * 64 + 32 * (lo8 ? 0 : 1) + 16 * (g & 1) + 8 * (g >> 1);
        const int rowA = m0 + wm * 128 + j * 16 + (mcol & 7);
        const bool okc = col < p.N;
        const unsigned oA = okc && rowA < p.M ? (unsigned)(((long)rowA * p.N + col) * 2) : 0x80000000u;
        const unsigned oB = okc && rowA + 8 < p.M ? (unsigned)(((long)(rowA + 8) * p.N + col) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(A, ry, oA, 0, 2);
        __builtin_amdgcn_raw_buffer_store_b128(B, ry, oB, 0, 2);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
}


// ---- staging-throughput probe: the w4 tile schedule with only the operand loads (timing only) ----
// RB: bytes of a row per load instruction (64: 16 rows x 64 B per 1-KiB piece; 128: 8 rows x 128 B);
// MODE 0: buffer_load ... lds; 1: buffer_load_dwordx4 into VGPRs (summed into a sink so they stay)
template <int RB, int MODE>
__global__ __launch_bounds__(256) void stage_probe_kernel(LabParams p, int tiles_m, int tiles_n, float* sink) {
  __shared__ __attribute__((aligned(1024))) h16 smem[4 * STAGE];
  int lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int ntiles = tiles_m * tiles_n;
  const int nk = p.K / BK;  // 32-deep steps: 32 KiB per step and CU either way
  const i4v xrs = rsrc4(p.x, (long)p.M * p.K * 2), wrs = rsrc4(p.w, (long)p.N * p.K * 2);
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(VDA_LDS h16*)smem);
  constexpr int RPP = 1024 / RB;        // rows per piece
  constexpr int LPR = RB / 16;          // lanes per row
  u32x4 acc = u32x4{0, 0, 0, 0};
  for (int vb = blockIdx.x; vb < ntiles; vb += gridDim.x) {
    int tm, tn;
    tile_coords(vb, ntiles, tiles_m, tiles_n, tm, tn);
    // RB = 64: 16 pieces per operand per step (rows 16q..); RB = 128: one step's bytes are 8 pieces of
    // 8 rows x 128 B per operand covering k 0..63 of 256 rows every other step (16 pieces per 2 steps)
    unsigned xo[8], wo[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = wave * 8 + i;  // 32 pieces of a 64-k stage per operand (RB = 128) / 16 per 32-k (RB = 64)
      const int r = (RB == 64 ? (q & 15) * 16 : q * 8) + lane / LPR;
      const int c = lane % LPR;
      const int m = tm * 256 + (r & 255), n = tn * 256 + (r & 255);
      xo[i] = m < p.M ? (unsigned)(((long)m * p.K + c * 8) * 2) : 0x80000000u;
      wo[i] = n < p.N ? (unsigned)(((long)n * p.K + c * 8) * 2) : 0x80000000u;
    }
    for (int t = 0; t < nk; ++t) {
      // per step and CU: 32 KiB = 32 pieces = 8 per wave (4 X + 4 W)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ii = RB == 64 ? i : (t & 1) * 4 + i;
        const int soff = RB == 64 ? t * BK * 2 : (t >> 1) * 128;
        if constexpr (MODE == 0) {
          dma16(xrs, xo[ii], soff, lds0 + (unsigned)(((t & 3) * 32 + wave * 8 + i) * 1024));
          dma16(wrs, wo[ii], soff, lds0 + (unsigned)(((t & 3) * 32 + wave * 8 + 4 + i) * 1024));
        } else {
          u32x4 a, b;
          asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(a) : "v"(xo[ii]), "s"(xrs), "s"(soff) : "memory");
          asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(b) : "v"(wo[ii]), "s"(wrs), "s"(soff) : "memory");
          asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
          acc += a ^ b;
        }
      }
      if constexpr (MODE == 0) wait_vm<24>();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc[0] == 0x12345678u && acc[1] == 7) sink[0] = 1.f;
}


// ---- w8: the product's 8-wave layout (2 m x 4 n waves, 128 x 64 wave tiles, 2 waves per SIMD) on the w4c
// pipeline: NST-stage BK=32 ring, one barrier per step, DMA / fragment reads / MFMAs placed by hand ----
template <int FL, int NST>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
void w8_kernel(LabParams p, int tiles_m, int tiles_n) {
  constexpr bool LB = NST * STAGE + 1024 <= 81920 && !(FL & 8);
  __shared__ __attribute__((aligned(1024))) h16 smem[NST * STAGE + (LB ? 1024 : 0)];
  constexpr int BOFS = NST * STAGE;
  int lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int ntiles = tiles_m * tiles_n;
  const int nk = p.K / BK;
  const i4v xrs = rsrc4(p.x, (long)p.M * p.K * 2), wrs = rsrc4(p.w, (long)p.N * p.K * 2);
  const i4v brs = rsrc4(p.bias, (long)p.N * 4);
  const int prow = lane >> 2;
  const int pch = (lane & 3) ^ swz(prow);
  const int frow = lane & 15, fch = lane >> 4;
  const unsigned fofs = (unsigned)(frow * BK + ((fch ^ swz(frow)) << 3)) * 2u;
  const unsigned xfo = fofs + (unsigned)(wm * 128 * BK * 2);
  const unsigned wfo = fofs + (unsigned)((256 + wn * 64) * BK * 2);
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(VDA_LDS h16*)smem);

  f4 acc[4][8];
  h8 fx[2][8], fw[2][4];
  int vb = blockIdx.x;
  unsigned xo[2], wo[2], bo = 0;
  int cnt = 0;
  auto offsets = [&](int vb_) {
    int tm, tn;
    tile_coords(vb_, ntiles, tiles_m, tiles_n, tm, tn);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (wave * 2 + i) * 16 + prow;
      const int m = tm * 256 + r, n = tn * 256 + r;
      xo[i] = m < p.M ? (unsigned)(((long)m * p.K + pch * 8) * 2) : 0x80000000u;
      wo[i] = n < p.N ? (unsigned)(((long)n * p.K + pch * 8) * 2) : 0x80000000u;
    }
    const int nb = tn * 256 + lane * 4;
    bo = nb < p.N ? (unsigned)(nb * 4) : 0x80000000u;
  };
  auto piece = [&](int t, int q) {  // piece q (0..3) of step t: X pieces 0-1, W pieces 2-3
    const unsigned sb = lds0 + (unsigned)((t % NST) * STAGE * 2);
    if (q < 2) dma16(xrs, xo[q], t * BK * 2, sb + (unsigned)((wave * 2 + q) * 1024));
    else dma16(wrs, wo[q - 2], t * BK * 2, sb + (unsigned)((256 * BK + (wave * 2 + q - 2) * 512) * 2));
  };
  auto prologue = [&](int slot) {
#pragma unroll
    for (int s = 0; s < NST; ++s)
#pragma unroll
      for (int q = 0; q < 4; ++q) piece(s, q);
    if (LB && wave == 0) dma16(brs, bo, 0, lds0 + (unsigned)((BOFS + slot * 512) * 2));
  };
  if (vb < ntiles) {
    offsets(vb);
    prologue(0);
  }
  for (; vb < ntiles; vb += gridDim.x, ++cnt) {
    int tm, tn;
    tile_coords(vb, ntiles, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    constexpr int YP = (NST - 1) * 4;
    if (vb == (int)blockIdx.x) {
      if (LB && wave == 0) wait_vm<YP + 1>(); else wait_vm<YP>();
    } else {
      if (LB && wave == 0) wait_vm<YP + 17>(); else wait_vm<YP + 16>();
    }
    __builtin_amdgcn_s_barrier();
    {
      const h16* sb = smem;
#pragma unroll
      for (int j = 0; j < 8; ++j) fx[0][j] = lds_frag(sb, xfo + j * 16 * BK * 2);
#pragma unroll
      for (int i = 0; i < 4; ++i) fw[0][i] = lds_frag(sb, wfo + i * 16 * BK * 2);
    }
    const int vb_next = vb + (int)gridDim.x;

    auto step = [&](int t, auto setc, auto waitc, auto dmac, auto readc, auto zc) {
      constexpr int S = decltype(setc)::value;
      constexpr int WAIT = decltype(waitc)::value;
      constexpr int DMA = decltype(dmac)::value;
      constexpr bool READ = decltype(readc)::value;
      constexpr bool Z = decltype(zc)::value;
      if constexpr (WAIT >= 0) wait_vm<WAIT>();
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
      if constexpr (DMA == 2) {
        if (vb_next < ntiles) {
          offsets(vb_next);
          prologue((cnt + 1) & 1);
        }
      }
      const h16* sb = smem + ((t + 1) % NST) * STAGE;
#pragma unroll
      for (int mi = 0; mi < 32; ++mi) {
        const int i = mi >> 3, j = mi & 7;
        if constexpr (FL & 2) {
          if (mi == 0) mfma_m(acc[i][j], fw[S][i], fx[S][j]);
        } else if constexpr (Z) mfma_z(acc[i][j], fw[S][i], fx[S][j]);
        else mfma_m(acc[i][j], fw[S][i], fx[S][j]);
        if constexpr (READ && !(FL & 4)) {
          if (mi % 2 == 0 && mi / 2 < 12) {
            const int r = mi / 2;
            if (r < 8) fx[S ^ 1][r] = lds_frag(sb, xfo + r * 16 * BK * 2);
            else fw[S ^ 1][r - 8] = lds_frag(sb, wfo + (r - 8) * 16 * BK * 2);
          }
        }
        if constexpr (DMA == 1 && !(FL & 1)) {
          if (mi % 8 == 3) piece(t + NST, mi / 8);
        }
      }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using WS = std::integral_constant<int, 4 * (NST - 2)>;
    using RT = std::integral_constant<bool, true>;
    using FT = std::false_type;
    step(0, I0{}, WS{}, I1{}, RT{}, std::true_type{});
    int t = 1;
    if constexpr (NST % 2 == 0) {
      step(1, I1{}, WS{}, I1{}, RT{}, FT{});
      t = 2;
      for (; t < nk - NST; t += 2) {
        step(t, I0{}, WS{}, I1{}, RT{}, FT{});
        step(t + 1, I1{}, WS{}, I1{}, RT{}, FT{});
      }
    } else {
      for (; t < nk - NST; t += 2) {
        step(t, I1{}, WS{}, I1{}, RT{}, FT{});
        step(t + 1, I0{}, WS{}, I1{}, RT{}, FT{});
      }
    }
    [&]<int... U>(std::integer_sequence<int, U...>) {
      (([&] {
         constexpr int u = U;
         using SU = std::integral_constant<int, (NST + u) & 1>;
         if constexpr (u == NST - 1) {
           step(nk - 1, SU{}, std::integral_constant<int, -1>{}, I2{}, std::false_type{}, FT{});
         } else {
           step(nk - NST + u, SU{}, std::integral_constant<int, 4 * (NST - u - 2 > 0 ? NST - u - 2 : 0)>{}, I0{}, RT{}, FT{});
         }
       }()), ...);
    }(std::make_integer_sequence<int, NST>{});
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

    const int mcol = lane & 15, g = lane >> 4;
    const bool lo8 = (mcol & 8) == 0;
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.y, (short)0, (int)((long)p.M * p.N * 2 < 0x7fffffffL ? (long)p.M * p.N * 2 : 0x7fffffffL), 0x00020000);
    f4 bv[4];
    {
      const float* bl = reinterpret_cast<const float*>(smem + BOFS + (cnt & 1) * 512);
#pragma unroll
      for (int i = 0; i < 4; ++i) bv[i] = LB ? *reinterpret_cast<const f4*>(bl + wn * 64 + i * 16 + g * 4) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      u32x4 o[2];
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int ia = 2 * pp;
        float a[4], c[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          a[r] = acc[ia][j][r] + bv[ia][r];
          c[r] = acc[ia + 1][j][r] + bv[ia + 1][r];
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
      const int col = n0 + wn * 64 + 32 * (lo8 ? 0 : 1) + 16 * (g & 1) + 8 * (g >> 1);
      const int rowA = m0 + wm * 128 + j * 16 + (mcol & 7);
      const bool okc = col < p.N;
      const unsigned oA = okc && rowA < p.M ? (unsigned)(((long)rowA * p.N + col) * 2) : 0x80000000u;
      const unsigned oB = okc && rowA + 8 < p.M ? (unsigned)(((long)(rowA + 8) * p.N + col) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(A, ry, oA, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b128(B, ry, oB, 0, 2);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
}

// ---- w8b: w8 with the MFMAs in X-block-major order, ONE X fragment set (each X fragment of step t+1 read
// right after the last MFMA of step t that uses its register) and two W sets: 64 fragment VGPRs instead of 96
// ---- (w8: the product's 8-wave layout (2 m x 4 n waves, 128 x 64 wave tiles, 2 waves per SIMD) on the w4c
// pipeline: NST-stage BK=32 ring, one barrier per step, DMA / fragment reads / MFMAs placed by hand ----
template <int FL, int NST>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
void w8b_kernel(LabParams p, int tiles_m, int tiles_n) {
  constexpr bool LB = NST * STAGE + 1024 <= 81920 && !(FL & 8);
  __shared__ __attribute__((aligned(1024))) h16 smem[NST * STAGE + (LB ? 1024 : 0)];
  constexpr int BOFS = NST * STAGE;
  int lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int ntiles = tiles_m * tiles_n;
  const int nk = p.K / BK;
  const i4v xrs = rsrc4(p.x, (long)p.M * p.K * 2), wrs = rsrc4(p.w, (long)p.N * p.K * 2);
  const i4v brs = rsrc4(p.bias, (long)p.N * 4);
  const int prow = lane >> 2;
  const int pch = (lane & 3) ^ swz(prow);
  const int frow = lane & 15, fch = lane >> 4;
  const unsigned fofs = (unsigned)(frow * BK + ((fch ^ swz(frow)) << 3)) * 2u;
  const unsigned xfo = fofs + (unsigned)(wm * 128 * BK * 2);
  const unsigned wfo = fofs + (unsigned)((256 + wn * 64) * BK * 2);
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(VDA_LDS h16*)smem);

  f4 acc[4][8];
  h8 fx[8], fw[2][4];
  int vb = blockIdx.x;
  unsigned xo[2], wo[2], bo = 0;
  int cnt = 0;
  auto offsets = [&](int vb_) {
    int tm, tn;
    tile_coords(vb_, ntiles, tiles_m, tiles_n, tm, tn);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (wave * 2 + i) * 16 + prow;
      const int m = tm * 256 + r, n = tn * 256 + r;
      xo[i] = m < p.M ? (unsigned)(((long)m * p.K + pch * 8) * 2) : 0x80000000u;
      wo[i] = n < p.N ? (unsigned)(((long)n * p.K + pch * 8) * 2) : 0x80000000u;
    }
    const int nb = tn * 256 + lane * 4;
    bo = nb < p.N ? (unsigned)(nb * 4) : 0x80000000u;
  };
  auto piece = [&](int t, int q) {  // piece q (0..3) of step t: X pieces 0-1, W pieces 2-3
    const unsigned sb = lds0 + (unsigned)((t % NST) * STAGE * 2);
    if (q < 2) dma16(xrs, xo[q], t * BK * 2, sb + (unsigned)((wave * 2 + q) * 1024));
    else dma16(wrs, wo[q - 2], t * BK * 2, sb + (unsigned)((256 * BK + (wave * 2 + q - 2) * 512) * 2));
  };
  auto prologue = [&](int slot) {
#pragma unroll
    for (int s = 0; s < NST; ++s)
#pragma unroll
      for (int q = 0; q < 4; ++q) piece(s, q);
    if (LB && wave == 0) dma16(brs, bo, 0, lds0 + (unsigned)((BOFS + slot * 512) * 2));
  };
  if (vb < ntiles) {
    offsets(vb);
    prologue(0);
  }
  for (; vb < ntiles; vb += gridDim.x, ++cnt) {
    int tm, tn;
    tile_coords(vb, ntiles, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    constexpr int YP = (NST - 1) * 4;
    if (vb == (int)blockIdx.x) {
      if (LB && wave == 0) wait_vm<YP + 1>(); else wait_vm<YP>();
    } else {
      if (LB && wave == 0) wait_vm<YP + 17>(); else wait_vm<YP + 16>();
    }
    __builtin_amdgcn_s_barrier();
    {
      const h16* sb = smem;
#pragma unroll
      for (int j = 0; j < 8; ++j) fx[j] = lds_frag(sb, xfo + j * 16 * BK * 2);
#pragma unroll
      for (int i = 0; i < 4; ++i) fw[0][i] = lds_frag(sb, wfo + i * 16 * BK * 2);
    }
    const int vb_next = vb + (int)gridDim.x;

    auto step = [&](int t, auto setc, auto waitc, auto dmac, auto readc, auto zc) {
      constexpr int S = decltype(setc)::value;
      constexpr int WAIT = decltype(waitc)::value;
      constexpr int DMA = decltype(dmac)::value;
      constexpr bool READ = decltype(readc)::value;
      constexpr bool Z = decltype(zc)::value;
      if constexpr (WAIT >= 0) wait_vm<WAIT>();
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
      if constexpr (DMA == 2) {
        if (vb_next < ntiles) {
          offsets(vb_next);
          prologue((cnt + 1) & 1);
        }
      }
      const h16* sb = smem + ((t + 1) % NST) * STAGE;
#pragma unroll
      for (int mi = 0; mi < 32; ++mi) {
        const int j = mi >> 2, i = mi & 3;  // X-block-major: fx[j] is dead after MFMA (j, 3)
        if constexpr (FL & 2) {
          if (mi == 0) mfma_m(acc[i][j], fw[S][i], fx[j]);
        } else if constexpr (Z) mfma_z(acc[i][j], fw[S][i], fx[j]);
        else mfma_m(acc[i][j], fw[S][i], fx[j]);
        if constexpr (READ && !(FL & 4)) {
          if (i == 3) fx[j] = lds_frag(sb, xfo + j * 16 * BK * 2);           // step t+1's X block j
          if (i == 1 && j < 4) fw[S ^ 1][j] = lds_frag(sb, wfo + j * 16 * BK * 2);  // step t+1's W block j
        }
        if constexpr (DMA == 1 && !(FL & 1)) {
          if (mi % 8 == 5) piece(t + NST, mi / 8);
        }
      }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using WS = std::integral_constant<int, 4 * (NST - 2)>;
    using RT = std::integral_constant<bool, true>;
    using FT = std::false_type;
    step(0, I0{}, WS{}, I1{}, RT{}, std::true_type{});
    int t = 1;
    if constexpr (NST % 2 == 0) {
      step(1, I1{}, WS{}, I1{}, RT{}, FT{});
      t = 2;
      for (; t < nk - NST; t += 2) {
        step(t, I0{}, WS{}, I1{}, RT{}, FT{});
        step(t + 1, I1{}, WS{}, I1{}, RT{}, FT{});
      }
    } else {
      for (; t < nk - NST; t += 2) {
        step(t, I1{}, WS{}, I1{}, RT{}, FT{});
        step(t + 1, I0{}, WS{}, I1{}, RT{}, FT{});
      }
    }
    [&]<int... U>(std::integer_sequence<int, U...>) {
      (([&] {
         constexpr int u = U;
         using SU = std::integral_constant<int, (NST + u) & 1>;
         if constexpr (u == NST - 1) {
           step(nk - 1, SU{}, std::integral_constant<int, -1>{}, I2{}, std::false_type{}, FT{});
         } else {
           step(nk - NST + u, SU{}, std::integral_constant<int, 4 * (NST - u - 2 > 0 ? NST - u - 2 : 0)>{}, I0{}, RT{}, FT{});
         }
       }()), ...);
    }(std::make_integer_sequence<int, NST>{});
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

    const int mcol = lane & 15, g = lane >> 4;
    const bool lo8 = (mcol & 8) == 0;
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.y, (short)0, (int)((long)p.M * p.N * 2 < 0x7fffffffL ? (long)p.M * p.N * 2 : 0x7fffffffL), 0x00020000);
    f4 bv[4];
    {
      const float* bl = reinterpret_cast<const float*>(smem + BOFS + (cnt & 1) * 512);
#pragma unroll
      for (int i = 0; i < 4; ++i) bv[i] = LB ? *reinterpret_cast<const f4*>(bl + wn * 64 + i * 16 + g * 4) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      u32x4 o[2];
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int ia = 2 * pp;
        float a[4], c[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          a[r] = acc[ia][j][r] + bv[ia][r];
          c[r] = acc[ia + 1][j][r] + bv[ia + 1][r];
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
      const int col = n0 + wn * 64 + 32 * (lo8 ? 0 : 1) + 16 * (g & 1) + 8 * (g >> 1);
      const int rowA = m0 + wm * 128 + j * 16 + (mcol & 7);
      const bool okc = col < p.N;
      const unsigned oA = okc && rowA < p.M ? (unsigned)(((long)rowA * p.N + col) * 2) : 0x80000000u;
      const unsigned oB = okc && rowA + 8 < p.M ? (unsigned)(((long)(rowA + 8) * p.N + col) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(A, ry, oA, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b128(B, ry, oB, 0, 2);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
}


// ---- w8r: register staging (buffer_load_dwordx4 -> VGPR -> ds_write_b128) of whole 128-B rows into a
// 2-stage [256][64]-half ring (the product's swizzle), 8 waves (2 m x 4 n, 128 x 64 wave tiles), one
// barrier per 64-deep step; MFMAs on AGPR accumulators (asm), X fragments rotated per block, two W sets.
// (The staging probe measured whole-row VGPR loads at ~1.3x the LDS-DMA rate.)
__device__ __forceinline__ unsigned swz64(int row, int chunk) {  // byte offset in a [rows][64 halves] image
  return (unsigned)(row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
}
template <int FL>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
void w8r_kernel(LabParams p, int tiles_m, int tiles_n) {
  constexpr int RS = 512 * 64;  // halves per stage (X 256 rows + W 256 rows of 64)
  __shared__ __attribute__((aligned(1024))) h16 smem[2 * RS];
  int lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int tid = wave * 64 + lane;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntiles = tiles_m * tiles_n;
  const int nk = p.K / 64;
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, (int)((long)p.M * p.K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, (int)((long)p.N * p.K * 2), 0x00020000);
  // staging: thread -> chunk c = tid & 7 of rows r0 + 64 i (i = 0..3), for X and for W
  const int c = tid & 7, r0 = tid >> 3;
  const unsigned lw = swz64(r0, c);  // + i * 8192 (row + 64: the swizzle term repeats every 16 rows)
  // fragments: row 16 blk + (lane & 15), 16-B chunk kh * 4 + (lane >> 4) of the 64-half row
  const int frow = lane & 15, fch = lane >> 4;
  unsigned fxo[2], fwo[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    fxo[kh] = swz64(wm * 128 + frow, kh * 4 + fch);
    fwo[kh] = (unsigned)(256 * 128) + swz64(wn * 64 + frow, kh * 4 + fch);
  }
  f4 acc[4][8];
  h8 fx[8], fw[2][4];
  u32x4 R[4];
  int vb = blockIdx.x;
  unsigned xo = 0, wo = 0;
  auto offsets = [&](int vb_) {
    int tm, tn;
    tile_coords(vb_, ntiles, tiles_m, tiles_n, tm, tn);
    const int m = tm * 256 + r0, n = tn * 256 + r0;
    xo = (unsigned)(((long)m * p.K + c * 8) * 2);
    wo = (unsigned)(((long)n * p.K + c * 8) * 2);
  };
  // the staging in two halves (X rows, then W rows; 16 VGPRs): each half is loaded, then written to the
  // next stage half a step later
  auto gload = [&](int t, int half) {  // rows past M / N: past num_records -> zeros
#pragma unroll
    for (int i = 0; i < 4; ++i)
      R[i] = __builtin_amdgcn_raw_buffer_load_b128(half ? wrs : xrs, half ? wo : xo, i * 64 * p.K * 2 + t * 128, 0);
  };
  auto lstore = [&](int stage, int half) {
    char* sb = reinterpret_cast<char*>(smem + stage * RS) + half * 256 * 128;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x4*>(sb + lw + i * 8192) = R[i];
  };
  const char* s0 = reinterpret_cast<const char*>(smem);
  auto xf = [&](int stage, int kh, int j) { return lds_frag(smem, stage * RS * 2 + fxo[kh] + j * 16 * 128); };
  auto wf = [&](int stage, int kh, int i) { return lds_frag(smem, stage * RS * 2 + fwo[kh] + i * 16 * 128); };
  (void)s0;
  if (vb < ntiles) {
    offsets(vb);
    gload(0, 0);
    lstore(0, 0);
    gload(0, 1);
  }
  for (; vb < ntiles; vb += gridDim.x) {
    int tm, tn;
    tile_coords(vb, ntiles, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int vb_next = vb + (int)gridDim.x;
    lstore(0, 1);  // step 0's second half (its first half was written by the previous tile's last step, or above)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    for (int t = 0; t < nk; ++t) {
      const int st = t & 1;
      const bool more = t + 1 < nk, chain = !more && vb_next < ntiles;
      if (more) gload(t + 1, 0);
      else if (chain) { offsets(vb_next); gload(0, 0); }
#pragma unroll
      for (int j = 0; j < 8; ++j) fx[j] = xf(st, 0, j);
#pragma unroll
      for (int i = 0; i < 4; ++i) fw[0][i] = wf(st, 0, i);
#pragma unroll
      for (int i = 0; i < 4; ++i) fw[1][i] = wf(st, 1, i);
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
        for (int mi = 0; mi < 32; ++mi) {
          const int j = mi >> 2, i = mi & 3;
          if constexpr (FL & 2) {
            if (mi == 0) mfma_m(acc[i][j], fw[kh][i], fx[j]);
          } else if (t == 0 && kh == 0) mfma_z(acc[i][j], fw[kh][i], fx[j]);
          else mfma_m(acc[i][j], fw[kh][i], fx[j]);
          if (kh == 0 && i == 3) fx[j] = xf(st, 1, j);  // X block j of k-half 1
        }
        if (kh == 0) {  // mid-step: the X half of the next step's rows goes to the other stage, W is requested
          if (more || chain) lstore(st ^ 1, 0);
          if (more) gload(t + 1, 1);
          else if (chain) gload(0, 1);
        }
      }
      if (more) lstore(st ^ 1, 1);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

    const int mcol = lane & 15, g = lane >> 4;
    const bool lo8 = (mcol & 8) == 0;
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.y, (short)0, (int)((long)p.M * p.N * 2 < 0x7fffffffL ? (long)p.M * p.N * 2 : 0x7fffffffL), 0x00020000);
    f4 bv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + wn * 64 + i * 16 + g * 4;
      bv[i] = n < p.N ? *reinterpret_cast<const f4*>(p.bias + n) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      u32x4 o[2];
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int ia = 2 * pp;
        float a[4], cc[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          a[r] = acc[ia][j][r] + bv[ia][r];
          cc[r] = acc[ia + 1][j][r] + bv[ia + 1][r];
          perm16_swap(a[r], cc[r]);
        }
        typedef float f2v __attribute__((ext_vector_type(2)));
        const h2 h0 = __builtin_convertvector(f2v{a[0], a[1]}, h2), h1 = __builtin_convertvector(f2v{a[2], a[3]}, h2);
        const h2 h2_ = __builtin_convertvector(f2v{cc[0], cc[1]}, h2), h3 = __builtin_convertvector(f2v{cc[2], cc[3]}, h2);
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
      const int col = n0 + wn * 64 + 32 * (lo8 ? 0 : 1) + 16 * (g & 1) + 8 * (g >> 1);
      const int rowA = m0 + wm * 128 + j * 16 + (mcol & 7);
      const bool okc = col < p.N;
      const unsigned oA = okc && rowA < p.M ? (unsigned)(((long)rowA * p.N + col) * 2) : 0x80000000u;
      const unsigned oB = okc && rowA + 8 < p.M ? (unsigned)(((long)(rowA + 8) * p.N + col) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(A, ry, oA, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b128(B, ry, oB, 0, 2);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
}


// ---- overlap probe (timing only, wrong output): does the LDS-DMA staging run beside the MFMA stream when
// waves that issue no MFMA issue it?  8 MFMA waves (2 per SIMD) run, per 32-deep K step, 12 ds_read_b128
// fragment reads of a fixed 32-KiB LDS image + 32 v_mfma_f32_16x16x32_f16 (the product's 128 x 64 wave
// tile), one barrier per step; the step's 32 KiB of X / W pieces (32 x 1 KiB) go into a 4-stage ring by
//   MODE 0: nobody (MFMA only)                      MODE 1: ND extra DMA waves, 32 / ND pieces each
//   MODE 2: the MFMA waves, 4 each (as the product) MODE 3: the DMA waves only (the MFMA waves just barrier)
//   MODE 5 / 6: as 1 / 0 with the MFMA operands in registers (no fragment reads: is the conflict the LDS?)
template <int MODE, int ND = 2, int WD = 1>
__global__ __launch_bounds__(512 + 64 * ND) void overlap_probe_kernel(LabParams p, int tiles_m, int tiles_n, float* sink) {
  __shared__ __attribute__((aligned(1024))) h16 smem[5 * STAGE];  // [0]: fragment image, [1..4]: the ring
  int lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const bool dmaw = wave >= 8;
  const int ntiles = tiles_m * tiles_n;
  const int nk = p.K / BK;
  const i4v xrs = rsrc4(p.x, (long)p.M * p.K * 2), wrs = rsrc4(p.w, (long)p.N * p.K * 2);
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(VDA_LDS h16*)smem);
  const int frow = lane & 15, fch = lane >> 4;
  const unsigned fofs = lds0 + (unsigned)(frow * BK + ((fch ^ swz(frow)) << 3)) * 2u + (unsigned)((wave & 1) * 128 * BK * 2);
  f4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
  for (int vb = blockIdx.x; vb < ntiles; vb += gridDim.x) {
    int tm, tn;
    tile_coords(vb, ntiles, tiles_m, tiles_n, tm, tn);
    // piece q of a step: operand q >> 4 (X, W), rows 16 (q & 15) + lane / 4, 16-B chunk lane & 3
    auto poff = [&](int q) {
      const int r = (q & 15) * 16 + (lane >> 2), c = lane & 3;
      const int row = (q >> 4) ? tn * 256 + r : tm * 256 + r;
      const int lim = (q >> 4) ? p.N : p.M;
      return row < lim ? (unsigned)(((long)row * p.K + c * 8) * 2) : 0x80000000u;
    };
    for (int t = 0; t < nk; ++t) {
      const unsigned ring = lds0 + (unsigned)((1 + (t & 3)) * STAGE * 2);
      if constexpr (MODE == 1 || MODE == 3 || MODE == 5) {
        if (dmaw) {  // DMA wave d: pieces d * PPD .. (X for the first half of the waves, W for the second);
                     // the row block in the scalar offset
          constexpr int PPD = 32 / ND;
          const int d = wave - 8, q0 = d * PPD;
          const unsigned vo = poff(q0 & 16);
#pragma unroll
          for (int j = 0; j < PPD; ++j)
            dma16((q0 >> 4) ? wrs : xrs, vo, t * BK * 2 + ((q0 & 15) + j) * 16 * p.K * 2, ring + (unsigned)(q0 + j) * 1024u);
          wait_vm<PPD * WD>();  // WD steps of pieces left in flight
        }
      }
      if constexpr (MODE == 2) {
        if (!dmaw) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int q = wave * 4 + j;
            dma16(q >> 4 ? wrs : xrs, poff(q), t * BK * 2, ring + (unsigned)q * 1024u);
          }
          wait_vm<4>();
        }
      }
      if constexpr (MODE != 3) {
        if (!dmaw) {
          h8 a[8], b[4];
          if constexpr (MODE >= 5) {  // operands from registers: no LDS traffic in the MFMA waves
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] = h8{(h16)(lane & 7), 0, 0, 0, 0, 0, 0, (h16)i};
#pragma unroll
            for (int i = 0; i < 4; ++i) b[i] = h8{(h16)(lane & 3), 0, 0, 0, 0, 0, 0, (h16)i};
#pragma unroll
            for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(a[i]));
#pragma unroll
            for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(b[i]));
          } else {
#pragma unroll
          for (int i = 0; i < 8; ++i)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[i]) : "v"(fofs), "n"(i * 16 * BK * 2));
#pragma unroll
          for (int i = 0; i < 4; ++i)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(b[i]) : "v"(fofs), "n"((256 + i * 16) * BK * 2));
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
#pragma unroll
          for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) mfma_m(acc[(mi * 4 + ni) & 7], a[mi], b[ni]);
        }
      }
      __builtin_amdgcn_s_barrier();
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  float sacc = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) sacc += acc[i][0];
  if (sacc == 1234.5f) sink[0] = sacc;
}
}  // namespace

extern "C" int lab_gemm(int variant, const void* x, const void* w, void* y, const float* bias, int M, int N, int K,
                        int grid, void* stream) {
  if (K % (2 * BK) != 0 || K < 8 * BK || N % 8 != 0 || M <= 0) return -22;
  LabParams p{(const h16*)x, (const h16*)w, (h16*)y, bias, M, N, K};
  const int tiles_m = (M + 255) / 256, tiles_n = (N + 255) / 256;
  const int nt = tiles_m * tiles_n;
  const int g = grid > 0 ? std::min(grid, nt) : std::min(nt, 256);
  hipStream_t st = (hipStream_t)stream;
  switch (variant) {
    case 0: hipLaunchKernelGGL(w4_kernel<0>, dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 1: hipLaunchKernelGGL(w4_kernel<1>, dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 2: hipLaunchKernelGGL(w4_kernel<2>, dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 3: hipLaunchKernelGGL(w4_kernel<3>, dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 4: hipLaunchKernelGGL((w4b_kernel<3, 8, 4>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 5: hipLaunchKernelGGL((w4b_kernel<2, 8, 4>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 6: hipLaunchKernelGGL((w4b_kernel<3, 4, 2>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 7: hipLaunchKernelGGL((w4b_kernel<3, 6, 16>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 20: hipLaunchKernelGGL((w4c_kernel<2, 8, 4, 0, 4>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 21: hipLaunchKernelGGL((w4c_kernel<2, 8, 4, 0, 5>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 22: hipLaunchKernelGGL((w4c_kernel<2, 8, 4, 6, 4>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 23: hipLaunchKernelGGL((w4c_kernel<2, 8, 4, 6, 5>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 24: hipLaunchKernelGGL((w4c_kernel<2, 8, 4, 8, 3>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 25: hipLaunchKernelGGL((w4c_kernel<2, 8, 4, 14, 3>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 30: hipLaunchKernelGGL((stage_probe_kernel<64, 0>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 31: hipLaunchKernelGGL((stage_probe_kernel<128, 0>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 32: hipLaunchKernelGGL((stage_probe_kernel<64, 1>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 33: hipLaunchKernelGGL((stage_probe_kernel<128, 1>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 40: hipLaunchKernelGGL((w8_kernel<0, 4>), dim3(g), dim3(512), 0, st, p, tiles_m, tiles_n); break;
    case 41: hipLaunchKernelGGL((w8_kernel<8, 5>), dim3(g), dim3(512), 0, st, p, tiles_m, tiles_n); break;
    case 42: hipLaunchKernelGGL((w8_kernel<6, 4>), dim3(g), dim3(512), 0, st, p, tiles_m, tiles_n); break;
    case 43: hipLaunchKernelGGL((w8_kernel<1, 4>), dim3(g), dim3(512), 0, st, p, tiles_m, tiles_n); break;
    case 44: hipLaunchKernelGGL((w8_kernel<5, 4>), dim3(g), dim3(512), 0, st, p, tiles_m, tiles_n); break;
    case 50: hipLaunchKernelGGL((w8b_kernel<0, 4>), dim3(g), dim3(512), 0, st, p, tiles_m, tiles_n); break;
    case 51: hipLaunchKernelGGL((w8b_kernel<8, 5>), dim3(g), dim3(512), 0, st, p, tiles_m, tiles_n); break;
    case 60: hipLaunchKernelGGL((w8r_kernel<0>), dim3(g), dim3(512), 0, st, p, tiles_m, tiles_n); break;
    case 62: hipLaunchKernelGGL((w8r_kernel<2>), dim3(g), dim3(512), 0, st, p, tiles_m, tiles_n); break;
    case 11: hipLaunchKernelGGL((w4b_kernel<2, 8, 4, 1>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 12: hipLaunchKernelGGL((w4b_kernel<2, 8, 4, 2>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 14: hipLaunchKernelGGL((w4b_kernel<2, 8, 4, 4>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 15: hipLaunchKernelGGL((w4b_kernel<2, 8, 4, 5>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 16: hipLaunchKernelGGL((w4b_kernel<2, 8, 4, 6>), dim3(g), dim3(256), 0, st, p, tiles_m, tiles_n); break;
    case 70: hipLaunchKernelGGL(overlap_probe_kernel<0>, dim3(g), dim3(640), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 71: hipLaunchKernelGGL(overlap_probe_kernel<1>, dim3(g), dim3(640), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 72: hipLaunchKernelGGL(overlap_probe_kernel<2>, dim3(g), dim3(640), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 73: hipLaunchKernelGGL(overlap_probe_kernel<3>, dim3(g), dim3(640), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 80: hipLaunchKernelGGL((overlap_probe_kernel<3, 4, 2>), dim3(g), dim3(768), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 81: hipLaunchKernelGGL((overlap_probe_kernel<3, 4, 3>), dim3(g), dim3(768), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 82: hipLaunchKernelGGL((overlap_probe_kernel<5, 4, 3>), dim3(g), dim3(768), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 83: hipLaunchKernelGGL((overlap_probe_kernel<1, 4, 3>), dim3(g), dim3(768), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 78: hipLaunchKernelGGL((overlap_probe_kernel<5, 2>), dim3(g), dim3(640), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 79: hipLaunchKernelGGL((overlap_probe_kernel<6, 2>), dim3(g), dim3(640), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 74: hipLaunchKernelGGL((overlap_probe_kernel<1, 4>), dim3(g), dim3(768), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 75: hipLaunchKernelGGL((overlap_probe_kernel<3, 4>), dim3(g), dim3(768), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 76: hipLaunchKernelGGL((overlap_probe_kernel<1, 8>), dim3(g), dim3(1024), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    case 77: hipLaunchKernelGGL((overlap_probe_kernel<3, 8>), dim3(g), dim3(1024), 0, st, p, tiles_m, tiles_n, (float*)y); break;
    default: return -22;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
