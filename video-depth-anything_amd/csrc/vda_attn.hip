// Spatial (DINOv2) and temporal (motion-module) attention, fp16 MFMA + fp32 online softmax.
#include "vda_common.h"
#include "../../include/vda.h"
#include <type_traits>
#include <stdlib.h>

#ifdef VDA_TS  // per-block clock stamps of the spatial attention (tools/clock_probe.py; experiments only)
__device__ unsigned long long g_atsc[8192][4];
#define ATSC(k) do { if (threadIdx.x == 0 && blockIdx.x < 8192) { \
    g_atsc[blockIdx.x][2 * (k)] = __builtin_amdgcn_s_memtime(); \
    g_atsc[blockIdx.x][2 * (k) + 1] = __builtin_amdgcn_s_memrealtime(); } } while (0)
extern "C" int vda_debug_attn_clock_stamps(void* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_atsc), sizeof(g_atsc), 0, hipMemcpyDeviceToHost);
}
#else
#define ATSC(k) do {} while (0)
#endif

namespace {

// =============================================================================================
// Spatial attention, D = 64.  Block = 4 waves x 32 queries = 128 queries of one (batch, head);
// key/value tiles of 64 rows are staged in LDS (register-staged double buffer).
//
// Everything is computed transposed so that a lane owns ONE query column:
//   Sᵀ = K · Qᵀ     (A = K rows from LDS, B = Q rows held in registers)   -> lane: 16 keys of q
//   Oᵀ += Vᵀ · Pᵀ   (A = Vᵀ via ds_read_b64_tr_b16 from the row-major V tile, B = P from regs)
// The Pᵀ accumulator feeds the PV MFMA directly: lane group g holds keys {4g..4g+3} of each
// 16-key subtile, so the PV k-order is permuted identically on the Vᵀ side (two tr reads per
// fragment, rows kc*32+4g.. and kc*32+16+4g..).  Oᵀ lanes hold 4 consecutive head channels of
// one query -> 8-byte output stores and per-lane softmax rescale, no cross-lane traffic except
// the 4-lane max/sum reductions.
// =============================================================================================
constexpr int SD = 64;       // head dim
constexpr int SQB = 128;     // queries per block
constexpr int SKB = 64;      // keys per tile

__device__ __forceinline__ int k_swz(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 1) & 7)) << 3); }
__device__ __forceinline__ int v_swz(int row, int chunk) { return row * 64 + ((chunk ^ (((row >> 1) & 3) << 1)) << 3); }

__global__ __launch_bounds__(256) void spatial_attn_kernel(const h16* __restrict__ qkv, h16* __restrict__ out,
                                                           int N, int H, float scale_log2) {
  __shared__ __attribute__((aligned(16))) h16 sK[2][SKB * SD];
  __shared__ __attribute__((aligned(16))) h16 sV[2][SKB * SD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = blockIdx.y, b = blockIdx.z;
  const int C = H * SD;
  const long ld = 3L * C;
  const h16* base = qkv + (long)b * N * ld;
  const int g = lane >> 4, li = lane & 15;

  // Q fragments (B operand), pre-scaled by scale*log2(e) so scores come out in log2 units:
  // lane holds Q[q = qs*16 + li][d = ks*32 + 8g .. +7]
  h8 qf[2][2];
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int q = blockIdx.x * SQB + wave * 32 + qs * 16 + li;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      h8 t = h8{0, 0, 0, 0, 0, 0, 0, 0};
      if (q < N) t = __builtin_bit_cast(h8, ldg16(base + (long)q * ld + h * SD + ks * 32 + g * 8));
#pragma unroll
      for (int e = 0; e < 8; ++e) t[e] = (h16)((float)t[e] * scale_log2);
      qf[qs][ks] = t;
    }
  }

  f4 o[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) o[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  float mrun[2] = {0.f, 0.f};
  // row sums ride on the PV MFMA: an extra 16-row "Vᵀ" block whose rows 0, 4, 8, 12 are ones puts
  // sum_k P[k][q] into register 0 of every lane group (no VALU adds, rescaled along with O)
  f4 lsum[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  const h16 one_or_zero = (lane & 3) == 0 ? (h16)1.f : (h16)0.f;
  const h8 ones = h8{one_or_zero, one_or_zero, one_or_zero, one_or_zero, one_or_zero, one_or_zero, one_or_zero, one_or_zero};
  bool first = true;

  // staging: each thread moves 2 K chunks and 2 V chunks (16 B) per tile
  const int srow = tid >> 3, schunk = tid & 7;
  uint4 rk[2], rv[2];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int key = kt * SKB + srow + 32 * i;
      if (key < N) {
        const h16* rp = base + (long)key * ld + h * SD + schunk * 8;
        rk[i] = ldg16(rp + C);
        rv[i] = ldg16(rp + 2 * C);
      } else {
        rk[i] = make_uint4(0, 0, 0, 0);
        rv[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<uint4*>(&sK[buf][k_swz(srow + 32 * i, schunk)]) = rk[i];
      *reinterpret_cast<uint4*>(&sV[buf][v_swz(srow + 32 * i, schunk)]) = rv[i];
    }
  };

  // one 64-key tile; MASK only for the last (partial) tile
  auto tile = [&](int kt, auto mask_tag) {
    constexpr bool MASK = decltype(mask_tag)::value;
    const int buf = kt & 1;
    // ---- Sᵀ = K Qᵀ : s[a][qs] lane holds keys a*16 + 4g + r, query qs*16 + li
    // the accumulators start at -m (running max, log2 units), so s = q.k*scale - m comes out of the
    // MFMA chain ready for exp2 (no per-score subtraction)
    f4 s[4][2];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) s[a][qs] = f4{-mrun[qs], -mrun[qs], -mrun[qs], -mrun[qs]};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const h8 kf = *reinterpret_cast<const h8*>(&sK[buf][k_swz(a * 16 + li, ks * 4 + g)]);
#pragma unroll
        for (int qs = 0; qs < 2; ++qs) s[a][qs] = mfma16(kf, qf[qs][ks], s[a][qs]);
      }
    }
    if constexpr (MASK) {
      const int kbase = kt * SKB;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kbase + a * 16 + 4 * g + r >= N) { s[a][0][r] = -INFINITY; s[a][1][r] = -INFINITY; }
    }
    // ---- online softmax (base 2); the O/l rescale is skipped when no row max grew (wave vote)
    h8 pf[2][2];  // [qs][kc] P fragments (B operand of PV)
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      // 16 scores -> 8 v_max3 (the file is built with -fno-honor-nans -mno-amdgpu-ieee, so no
      // canonicalising v_max on the MFMA results), then the 4 lane groups via permlane swaps
      float mx = fmaxf(fmaxf(s[0][qs][0], s[0][qs][1]), s[0][qs][2]);
      mx = fmaxf(fmaxf(mx, s[0][qs][3]), s[1][qs][0]);
      mx = fmaxf(fmaxf(mx, s[1][qs][1]), s[1][qs][2]);
      mx = fmaxf(fmaxf(mx, s[1][qs][3]), s[2][qs][0]);
      mx = fmaxf(fmaxf(mx, s[2][qs][1]), s[2][qs][2]);
      mx = fmaxf(fmaxf(mx, s[2][qs][3]), s[3][qs][0]);
      mx = fmaxf(fmaxf(mx, s[3][qs][1]), s[3][qs][2]);
      mx = fmaxf(mx, s[3][qs][3]);
      mx = group_max4(mx);
      // mx is the tile max relative to the running max.  Deferred rescale (T13): keep the stale
      // max while mx <= 8, i.e. P <= 2^8, exact in fp16 P / fp32 sums.  The first tile always
      // re-bases (m starts at 0, not at a real max).
      if (first || __any(mx > 8.f)) {
        const float sh = first ? mx : fmaxf(mx, 0.f);
        const float alpha = __builtin_amdgcn_exp2f(-sh);
        mrun[qs] += sh;
        lsum[qs][0] *= alpha;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d][qs] *= alpha;
#pragma unroll
        for (int a = 0; a < 4; ++a) s[a][qs] -= sh;
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) pf[qs][a >> 1][(a & 1) * 4 + r] = (h16)__builtin_amdgcn_exp2f(s[a][qs][r]);
    }
    // ---- Oᵀ += Vᵀ Pᵀ
    const int q4 = li >> 2, p4 = li & 3;
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        // lane 4q+p of group g: row kc*32 + 4g + q, cols d*16 + 4p
        const int col = d * 16 + 4 * p4;
        const int r0 = kc * 32 + 4 * g + q4, r1 = r0 + 16;
        const h4 v0 = lds_read_tr16(&sV[buf][v_swz(r0, col >> 3) + (col & 7)]);
        const h4 v1 = lds_read_tr16(&sV[buf][v_swz(r1, col >> 3) + (col & 7)]);
        const h8 vf = h8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
        for (int qs = 0; qs < 2; ++qs) o[d][qs] = mfma16(vf, pf[qs][kc], o[d][qs]);
      }
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) lsum[qs] = mfma16(ones, pf[qs][kc], lsum[qs]);
    }
  };

  const int ntiles = (N + SKB - 1) / SKB;
  const int nfull = N / SKB;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    if (kt + 1 < ntiles) gload(kt + 1);
    if (kt < nfull) tile(kt, std::false_type{});
    else tile(kt, std::true_type{});
    first = false;
    if (kt + 1 < ntiles) sstore((kt + 1) & 1);
    __syncthreads();
  }
  // ---- epilogue: normalise and store (lane: d = dsub*16 + 4g + r, q = qs*16 + li)
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const float inv = 1.f / lsum[qs][0];
    const int q = blockIdx.x * SQB + wave * 32 + qs * 16 + li;
    if (q < N) {
      h16* op = out + ((long)b * N + q) * C + h * SD;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        h4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (h16)(o[d][qs][r] * inv);
        *reinterpret_cast<h4*>(op + d * 16 + 4 * g) = v;
      }
    }
  }
}

// =============================================================================================
// Spatial attention, D = 64, v_mfma_f32_32x32x16_f16 (the 32-cycle MFMA leaves 24 issue cycles per
// gap for the softmax VALU, the 16x16x32 one only 8).  Block = 4 waves x 32 queries of one (batch,
// head); a wave owns 32 query columns, a lane q = lane & 31 and half hf = lane >> 5.
//   Sᵀ[key][q] = K·Qᵀ   A = K rows (LDS, ds_read_b128), B = Q (registers, pre-scaled by scale·log2e);
//                       the chain starts from C = -m (a 16-register tile of the running reference
//                       m, see the deferred re-base below), so the scores come out relative to it
//                       with no VALU subtraction.
//   Oᵀ += Vᵀ·Pᵀ         B = P straight from the Sᵀ registers (k order 16st + 8(j>>2) + 4hf + (j&3)),
//                       A = Vᵀ by ds_read_b64_tr_b16 in the same permuted key order.
// K/V tiles (64 keys x 64 channels, 8 KiB each) arrive by LDS-DMA (4 x 1-KiB pieces per wave per
// tile, keys >= N read as zeros) into a 2-slot ring, one barrier per tile.  The softmax unit is a
// 32-key half of the tile: its 4 QK MFMAs, 16 exponentials and 4 PV MFMAs, so only half a tile of
// scores / P is live: 119 VGPRs, FOUR waves per SIMD (4 blocks x 32 KiB of LDS per CU), which cover
// each other's LDS / MFMA / exp latency chains better than three waves of whole-tile work (152 VGPRs).
// The two ring slots are two __shared__ objects and the tile loop is unrolled by 2 with static slots:
// with one ring array hipcc cannot prove that a tile's V reads do not alias the DMA in flight into the
// other slot and drains it (s_waitcnt vmcnt(0)) before every tile's first V read.  s_setprio 1 around
// the MFMA clusters lets a wave that reaches its MFMAs issue them ahead of the other waves' softmax VALU.
// The block -> (b, h, query block) map keeps all query blocks of one (b, h) on one XCD (K/V re-reads
// hit that L2).  LDS images: K slot row*8 + (chunk ^ ((row >> 1) & 7)), V slot row*8 + (chunk ^
// (((row >> 1) & 1) << 2)): conflict-free for the b128 K reads and the b64 transposed V reads.
// Measured (tools/ab_attn.py, same box, ViT-L 32 x 1370 x 16): whole-tile softmax, 3-slot ring, three
// waves per SIMD (round 5) 292-298 us; halves at three waves per SIMD 297; halves + 4 waves/SIMD 282-289;
// + static slots 276; + s_setprio 272-275 (r06_ab_attn_*.log).  Rejected: 8-wave blocks (297-302),
// row sums by v_dot2 on the packed P (+3 %), the half's K reads issued ahead of the chain (no change),
// and a software-pipelined wave (the next half's QK chain issued under the current half's softmax,
// 3-slot ring, 2 / 3 waves per SIMD: 343 / 330 us, bit-identical: profiles/r06_ab_attn_pipe.log).
// Earlier rounds: QK of tile t+1 before the softmax of tile t 333 vs 292 us; two 32-query sets per
// wave 317.8 / 307.8 vs 275.0 us (r05_ab_attn_two_sets.log).
// =============================================================================================
constexpr int SA_KT = 64;    // keys per tile

__device__ __forceinline__ int sa_kslot(int row, int c) { return row * 8 + (c ^ ((row >> 1) & 7)); }
__device__ __forceinline__ int sa_vslot(int row, int c) { return row * 8 + (c ^ (((row >> 1) & 1) << 2)); }
__global__ __launch_bounds__(256, 4) void spatial_attn32_kernel(const h16* __restrict__ qkv, h16* __restrict__ out,
                                                                int N, int H, int nqb, int nblocks, float scale_log2) {
  __shared__ __attribute__((aligned(16))) h16 sKV0[2][SA_KT * SD];  // ring slot 0: [K | V]
  __shared__ __attribute__((aligned(16))) h16 sKV1[2][SA_KT * SD];  // ring slot 1
  ATSC(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int id = blockIdx.x;
  const int per = nblocks >> 3;
  if (id < per * 8) id = (id & 7) * per + (id >> 3);
  const int qb = __builtin_amdgcn_readfirstlane(id % nqb), bh = id / nqb;  // scalar (the buffer
  const int h = __builtin_amdgcn_readfirstlane(bh % H), b = __builtin_amdgcn_readfirstlane(bh / H);  // rsrc)
  const int C = H * SD;
  const long ld = 3L * C;
  const h16* base = qkv + (long)b * N * ld + h * SD;
  const int r32 = lane & 31, hf = lane >> 5;
  const int q = qb * 128 + wave * 32 + r32;

  h8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    h8 t = h8{0, 0, 0, 0, 0, 0, 0, 0};
    if (q < N) t = __builtin_bit_cast(h8, ldg16(base + (long)q * ld + ks * 16 + hf * 8));
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = (h16)((float)t[e] * scale_log2);
    qf[ks] = t;
  }

  // 16 pieces per tile (8 K + 8 V, 8 key rows each); wave w moves pieces 4w .. 4w+3.  Buffer loads
  // with the (b, h) rows as the record range: keys >= N read as zeros.  Per-lane offsets are fixed
  // across tiles (the tile advances by the scalar offset).
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)((long)N * ld * 2), 0x00020000);
  unsigned voff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int gp = wave * 4 + j, isv = gp >> 3, pc = gp & 7;
    const int slot = pc * 64 + lane, row = slot >> 3, pos = slot & 7;
    const int c = isv ? (pos ^ (((row >> 1) & 1) << 2)) : (pos ^ ((row >> 1) & 7));
    voff[j] = (unsigned)(((long)row * ld + (isv ? 2 * C : C) + c * 8) * 2);
  }
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  // slot as a compile-time constant (the unrolled loop) or a run-time int (the tiles outside it)
  auto slot_ptr = [&](auto sl, int isv) -> h16* {
    if constexpr (std::is_same<decltype(sl), int>::value) return sl ? sKV1[isv] : sKV0[isv];
    else return decltype(sl)::value == 0 ? sKV0[isv] : sKV1[isv];
  };
  auto dma = [&](int kt, auto sl) {  // tile kt -> ring slot sl (= kt & 1)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int gp = wave * 4 + j, isv = gp >> 3, pc = gp & 7;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(krs, (VDA_LDS void*)(slot_ptr(sl, isv) + pc * 512), 16, (int)voff[j],
                                               (int)(kt * SA_KT * ld * 2), 0, 0);
    }
  };

  f16x o[2] = {f16x{}, f16x{}};
  f16x negm = {};
  float mrun = 0.f, lsum = 0.f;
  const int grp = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;

  // Lane-constant LDS byte offsets: K fragment ks of key row r32 (key block kb adds 32 rows = 4 KiB),
  // transposed-V read base of output tile dt (key slice ps adds 16 rows = 2 KiB, the second read of
  // a fragment 8 rows = 1 KiB).  The swizzle terms depend on the lane only, so the reads cost one
  // address add per ks / dt and the rest are immediate offsets.
  unsigned kofs[4], vofs[2];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) kofs[ks] = (unsigned)sa_kslot(r32, ks * 2 + hf) * 16u;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const int col = dt * 32 + (grp & 1) * 16 + 4 * p4, r0 = 4 * (grp >> 1) + q4;
    vofs[dt] = (unsigned)(sa_vslot(r0, col >> 3) * 8 + (col & 7)) * 2u;
  }
  // Deferred re-base (FA-style online softmax without a per-tile max): P = exp2(S - m) against the
  // running reference m; a half only re-bases when a lane's P sum passes 2^15 (then some P may not fit
  // fp16: the scores are recomputed, the true max taken and the half redone), so the steady state
  // computes no max at all.  P <= 2^15 keeps P exact to fp16 rounding and the fp32 sums far from
  // overflow.  The first half of the first tile always re-bases (m starts at 0, not at a real max).
  auto tile = [&](int kt, auto first_tag, auto mask_tag, auto sl) {
    constexpr bool FIRST = decltype(first_tag)::value;
    constexpr bool MASK = decltype(mask_tag)::value;
    const char* kbase = reinterpret_cast<const char*>(slot_ptr(sl, 0));
    const char* vbase = reinterpret_cast<const char*>(slot_ptr(sl, 1));
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      f16x s1;
      auto qk = [&]() {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const h8 kf = *reinterpret_cast<const h8*>(kbase + kofs[ks] + kb * 4096);
          s1 = mfma32(kf, qf[ks], ks == 0 ? negm : s1);
        }
        if constexpr (MASK) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kt * SA_KT + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf >= N) s1[r] = -INFINITY;
        }
      };
      auto smax = [&]() {
        float mx = fmaxf(fmaxf(s1[0], s1[1]), s1[2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) mx = fmaxf(fmaxf(mx, s1[r]), s1[r + 1]);
        mx = fmaxf(mx, s1[15]);
        return half_max(mx);
      };
      auto rebase = [&](float sh) {
        mrun += sh;
#pragma unroll
        for (int r = 0; r < 16; ++r) negm[r] = -mrun;
        s1 -= sh;
      };
      h8 pf[2];
      float tt;
      auto expo = [&]() {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = __builtin_amdgcn_exp2f(s1[r]);
          tt = r == 0 ? pv : tt + pv;  // (no add of 0 to start the chain)
          pf[r >> 3][r & 7] = (h16)pv;
        }
      };
      __builtin_amdgcn_s_setprio(1);
      qk();
      __builtin_amdgcn_s_setprio(0);
      if (FIRST && kb == 0) {
        rebase(smax());
        expo();
      } else {
        expo();
        if (__any(!(tt <= 32768.f))) {  // rare: re-base this half on its true max and redo it
          qk();  // the scores again (the K slot is still resident): they need not stay live past expo
          const float sh = fmaxf(smax(), 0.f);
          const float alpha = __builtin_amdgcn_exp2f(-sh);
          lsum *= alpha;
          o[0] *= alpha;
          o[1] *= alpha;
          rebase(sh);
          expo();
        }
      }
      lsum += tt;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ps = 0; ps < 2; ++ps) {  // the two output tiles' chains interleaved
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const char* va = vbase + vofs[dt] + (kb * 2 + ps) * 2048;
          const h4 v0 = lds_read_tr16(reinterpret_cast<const h16*>(va));
          const h4 v1 = lds_read_tr16(reinterpret_cast<const h16*>(va + 1024));
          const h8 vf = h8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
          o[dt] = mfma32(vf, pf[ps], o[dt]);
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
  };
  const int ntiles = (N + SA_KT - 1) / SA_KT;
  // tile kt landed and visible (its DMA is this wave's only one in flight), and every wave is done with
  // tile kt - 1: its slot takes tile kt + 1
  auto enter = [&](int kt, auto next_slot) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), as the builtin: hipcc's own wait bookkeeping sees it
    __builtin_amdgcn_s_barrier();
    if (kt + 1 < ntiles) dma(kt + 1, next_slot);
  };
  // a tile whose slot is only known at run time (the first, an odd leftover and the partial last one)
  auto tile_any = [&](int kt, auto first_tag, auto mask_tag) {
    enter(kt, (kt + 1) & 1);
    tile(kt, first_tag, mask_tag, kt & 1);
  };
  dma(0, S0{});
  const bool tail = N % SA_KT != 0;
  if (ntiles == 1 && tail) tile_any(0, std::true_type{}, std::true_type{});
  else tile_any(0, std::true_type{}, std::false_type{});
  const int nfull = ntiles - (tail ? 1 : 0);
  int kt = 1;
  for (; kt + 1 < nfull; kt += 2) {  // pairs: odd kt in slot 1, even kt + 1 in slot 0
    enter(kt, S0{});
    tile(kt, std::false_type{}, std::false_type{}, S1{});
    enter(kt + 1, S1{});
    tile(kt + 1, std::false_type{}, std::false_type{}, S0{});
  }
  if (kt < nfull) tile_any(kt, std::false_type{}, std::false_type{});
  if (tail && ntiles > 1) tile_any(ntiles - 1, std::false_type{}, std::true_type{});
  // epilogue: lane holds Oᵀ[d = dt*32 + 8gq + 4hf + r][q]
  const float inv = 1.f / half_sum(lsum);
  if (q < N) {
    h16* op = out + ((long)b * N + q) * C + h * SD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        h4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (h16)(o[dt][gq * 4 + r] * inv);
        *reinterpret_cast<h4*>(op + dt * 32 + 8 * gq + 4 * hf) = v;
      }
  }
  ATSC(1);
}

// =============================================================================================
// Temporal attention: one wave per (batch, site s, head), T <= 32 frames, v_mfma_f32_32x32x16_f16.
//   Sᵀ[key][q] = Σ_d K[key][d] Q[q][d]       A = K rows, B = Q rows (fragments straight from HBM)
//   Oᵀ[d][q]   = Σ_key Vᵀ[d][key] Pᵀ[key][q]  B = Pᵀ accumulator registers 8s..8s+7 (k order
//                16s + 8(j>>2) + 4h + (j&3)), A = Vᵀ by ds_read_b64_tr_b16 from a per-wave V tile.
// DP = head dim padded to a multiple of 16 (zero-filled), NDT = 32-wide output d tiles.
// =============================================================================================
// pe='rope' (attention.py:403-429): rotate the 4 channel pairs of an 8-channel q and k fragment of
// frame t, first channel c0 (even) of C: angle t * theta^(-2i/C) for pair i, fp32 math on the fp16
// values (the reference's q.float() complex multiply, type_as back to fp16)
__device__ __forceinline__ void rope_frag(h8& q, h8& k, int t, int c0, int C, float theta) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = (c0 >> 1) + j;
    const float freq = 1.f / powf(theta, (float)(2 * i) / (float)C);
    float sn, cs;
    sincosf((float)t * freq, &sn, &cs);
    const float qa = (float)q[2 * j], qb = (float)q[2 * j + 1];
    const float ka = (float)k[2 * j], kb = (float)k[2 * j + 1];
    q[2 * j] = (h16)(qa * cs - qb * sn);
    q[2 * j + 1] = (h16)(qa * sn + qb * cs);
    k[2 * j] = (h16)(ka * cs - kb * sn);
    k[2 * j + 1] = (h16)(ka * sn + kb * cs);
  }
}

__device__ __attribute__((aligned(64))) uint4 g_ta_zero[4];

constexpr int VDA_TA_NW = 4;  // waves (heads of one site) per temporal-attention block
template <int DP>
__global__ __launch_bounds__(64 * VDA_TA_NW) void temporal_attn_kernel(const h16* __restrict__ qkv, h16* __restrict__ out,
                                                            int B, int T, int S, int H, int D, float scale_log2,
                                                            float rope_theta) {
  constexpr int NST = DP / 16;
  constexpr int NDT = (DP + 31) / 32;
  constexpr int DP32 = NDT * 32;
  constexpr int VSTR = DP32 + (DP32 > 32 ? 32 : 0);  // row stride (halfs) of the V tile
  __shared__ __attribute__((aligned(16))) h16 sV[VDA_TA_NW][32 * VSTR];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long item = (long)blockIdx.x * VDA_TA_NW + wave;
  const long nitems = (long)B * S * H;
  const bool active = item < nitems;
  const int hh = active ? (int)(item % H) : 0;
  const long bs = active ? item / H : 0;
  const int s = (int)(bs % S), b = (int)(bs / S);
  const int C = H * D;
  const long ld = 3L * C;
  const int r32 = lane & 31, hf = lane >> 5;
  h16* vt = sV[wave];

  // V tile -> LDS (rows = keys, zero beyond T / D)
  {
    constexpr int CPR = DP32 / 8;  // 16-B chunks per row
    for (int i = lane; i < 32 * CPR; i += 64) {
      const int key = i / CPR, ch = i - key * CPR;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (active && key < T && ch * 8 < D)
        v = ldg16(qkv + ((long)(b * T + key) * S + s) * ld + 2 * C + hh * D + ch * 8);
      *reinterpret_cast<uint4*>(vt + key * VSTR + ch * 8) = v;
    }
  }
  // Sᵀ
  f16x acc = {};
  const long krow = ((long)(b * T + r32) * S + s) * ld + hh * D;
#pragma unroll
  for (int st = 0; st < NST; ++st) {
    const int d0 = st * 16 + hf * 8;
    h8 kf = h8{0, 0, 0, 0, 0, 0, 0, 0}, qf = kf;
    if (active && r32 < T && d0 < D) {
      qf = __builtin_bit_cast(h8, ldg16(qkv + krow + d0));
      kf = __builtin_bit_cast(h8, ldg16(qkv + krow + C + d0));
      if (rope_theta > 0.f) rope_frag(qf, kf, r32, hh * D + d0, C, rope_theta);
    }
    acc = mfma32(kf, qf, acc);
  }
  // softmax over keys (lane holds keys (r&3)+8(r>>2)+4hf for query r32; partner lane^32 the rest)
  float mx = -INFINITY;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int key = (r & 3) + 8 * (r >> 2) + 4 * hf;
    float t = acc[r] * scale_log2;
    if (key >= T) t = -INFINITY;
    acc[r] = t;
    mx = fmaxf(mx, t);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
  h8 pf[2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float p = exp2f(acc[r] - mx);
    sum += p;
    pf[r >> 3][r & 7] = (h16)p;
  }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;
  __syncthreads();  // V tile visible to the whole wave (all waves reach this)

  const int grp = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    f16x o = {};
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      // tr16 read: group grp -> key rows 16st + 4*(grp>>1) + q4 (+8), cols dt*32 + (grp&1)*16 + 4p4
      const int col = dt * 32 + (grp & 1) * 16 + 4 * p4;
      const int r0 = 16 * st + 4 * (grp >> 1) + q4;
      const h4 v0 = lds_read_tr16(vt + r0 * VSTR + col);
      const h4 v1 = lds_read_tr16(vt + (r0 + 8) * VSTR + col);
      const h8 vf = h8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      o = mfma32(vf, pf[st], o);
    }
    // lane holds Oᵀ[d = dt*32 + (r&3) + 8(r>>2) + 4hf][q = r32]
    if (active && r32 < T) {
      h16* op = out + ((long)(b * T + r32) * S + s) * C + hh * D;
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d = dt * 32 + 8 * gq + 4 * hf;
        if (d < D) {
          h4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (h16)(o[gq * 4 + r] * inv);
          *reinterpret_cast<h4*>(op + d) = v;
        }
      }
    }
  }
}

// Temporal attention with the (site, head)'s q, k and v rows staged in LDS (north_star; verdict r1
// item 10).  The direct-load kernel above reads its K / Q fragments as 32-B pieces of 32 different
// frame rows per instruction (rows S * 3C apart), which held it at ~3.5 TB/s.  Here each wave moves
// its head's three 32 x D tiles into LDS with global_load_lds, 16 B per lane, whole D*2-B row
// segments per 16 / 4 / 2 lanes (D = 128 / 64 / 32), then reads the MFMA fragments from LDS.  LDS
// image: row r of a tile = D halfs, 16-B chunk c at position c ^ ((r / (16 / CH)) & (CH - 1)),
// CH = D / 8: conflict-free for the K / Q fragment reads (ds_read_b128 lane groups = 16 rows of one
// chunk).  The output goes back through the q tile so it is stored as whole row segments too.
// Waves never share LDS, so the only sync is each wave's own vmcnt + one block barrier.
template <int D, int NW>
__global__ __launch_bounds__(64 * NW) void temporal_attn_lds_kernel(const h16* __restrict__ qkv, h16* __restrict__ out,
                                                                  int B, int T, int S, int H, float scale_log2,
                                                                  float rope_theta) {
  constexpr int CH = D / 8;                 // 16-B chunks per row
  constexpr int RPG = 16 / CH;              // rows per 256-B bank line
  constexpr int TILE = 32 * D;              // halfs per tensor tile
  constexpr int NI = 32 * CH / 64;          // DMA instructions per tensor
  constexpr int NST = D / 16;
  constexpr int NDT = D / 32;
  __shared__ __attribute__((aligned(16))) h16 sm[NW * 3 * TILE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long item = (long)blockIdx.x * NW + wave;
  const long nitems = (long)B * S * H;
  const bool active = item < nitems;
  const int hh = active ? (int)(item % H) : 0;
  const long bs = active ? item / H : 0;
  const int s = (int)(bs % S), b = (int)(bs / S);
  const int C = H * D;
  const long ld = 3L * C;
  h16* tq = sm + wave * 3 * TILE;
  h16* tk = tq + TILE;
  h16* tv = tk + TILE;
  auto pos = [](int row, int c) { return c ^ ((row / RPG) & (CH - 1)); };

  // stage q, k, v: slot sl = i * 64 + lane of a tile holds row sl / CH, chunk pos(row, sl % CH)
#pragma unroll
  for (int z = 0; z < 3; ++z) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int sl = i * 64 + lane;
      const int row = sl / CH;
      const int c = pos(row, sl % CH);
      const void* src = g_ta_zero;
      if (active && row < T) src = qkv + ((long)(b * T + row) * S + s) * ld + z * C + hh * D + c * 8;
      __builtin_amdgcn_global_load_lds(src, (VDA_LDS void*)(tq + z * TILE + i * 512), 16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // Sᵀ = K Qᵀ: lane (r32, hf) holds K / Q row r32, channels st * 16 + hf * 8 .. + 7
  const int r32 = lane & 31, hf = lane >> 5;
  f16x acc = {};
#pragma unroll
  for (int st = 0; st < NST; ++st) {
    const int c = st * 2 + hf;
    h8 kf = *reinterpret_cast<const h8*>(tk + r32 * D + pos(r32, c) * 8);
    h8 qf = *reinterpret_cast<const h8*>(tq + r32 * D + pos(r32, c) * 8);
    if (rope_theta > 0.f) rope_frag(qf, kf, r32, hh * D + c * 8, C, rope_theta);
    acc = mfma32(kf, qf, acc);
  }
  // softmax over keys (lane holds keys (r&3)+8(r>>2)+4hf for query r32; partner lane^32 the rest);
  // rows >= T are zero in LDS and masked here
  float mx = -INFINITY;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int key = (r & 3) + 8 * (r >> 2) + 4 * hf;
    float t = acc[r] * scale_log2;
    if (key >= T) t = -INFINITY;
    acc[r] = t;
    mx = fmaxf(mx, t);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
  h8 pf[2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float p = exp2f(acc[r] - mx);
    sum += p;
    pf[r >> 3][r & 7] = (h16)p;
  }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;

  const int grp = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    f16x o = {};
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      // tr16 read: group grp -> key rows 16st + 4*(grp>>1) + q4 (+8), cols dt*32 + (grp&1)*16 + 4p4
      const int col = dt * 32 + (grp & 1) * 16 + 4 * p4;
      const int r0 = 16 * st + 4 * (grp >> 1) + q4;
      const h4 v0 = lds_read_tr16(tv + r0 * D + pos(r0, col >> 3) * 8 + (col & 7));
      const h4 v1 = lds_read_tr16(tv + (r0 + 8) * D + pos(r0 + 8, col >> 3) * 8 + (col & 7));
      const h8 vf = h8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      o = mfma32(vf, pf[st], o);
    }
    // lane holds Oᵀ[d = dt*32 + (r&3) + 8(r>>2) + 4hf][q = r32]: into the q tile (its fragments are
    // consumed) as rows, so the stores below write whole D*2-B row segments
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int d = dt * 32 + 8 * gq + 4 * hf;
      h4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (h16)(o[gq * 4 + r] * inv);
      *reinterpret_cast<h4*>(tq + r32 * D + pos(r32, d >> 3) * 8 + (d & 7)) = v;
    }
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int sl = i * 64 + lane;
    const int row = sl / CH, c = sl % CH;
    const uint4 v = *reinterpret_cast<const uint4*>(tq + row * D + pos(row, c) * 8);
    if (active && row < T) *reinterpret_cast<uint4*>(out + ((long)(b * T + row) * S + s) * C + hh * D + c * 8) = v;
  }
}

// vda_debug_attn (tuning build): the round-1 spatial kernel / the direct-load temporal kernel
VDA_KNOB(int, g_sa_old, 0);
VDA_KNOB(int, g_ta_old, 0);

}  // namespace

#ifdef VDA_TUNING
extern "C" int vda_debug_attn(int32_t spatial_old, int32_t temporal_old) {
  g_sa_old = spatial_old;
  g_ta_old = temporal_old;
  return 0;
}
#endif

extern "C" int vda_spatial_attention(const void* qkv, void* out, int32_t B, int32_t N, int32_t H,
                                     int32_t D, float scale, void* stream) {
  VDA_CHECK_ARG(qkv && out, "null pointer");
  VDA_CHECK_ARG(B > 0 && N > 0 && H > 0, "empty attention");
  VDA_CHECK_ARG(D == SD, "spatial attention supports head dim 64 only");
  if (g_sa_old) {
    dim3 grid((N + SQB - 1) / SQB, H, B);
    hipLaunchKernelGGL(spatial_attn_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const h16*)qkv,
                       (h16*)out, N, H, scale * 1.4426950408889634f);
  } else {
    const int nqb = (N + 127) / 128;
    const long nb = (long)nqb * H * B;
    VDA_CHECK_ARG(nb < 0x7fffffffL, "attention grid too large");
    hipLaunchKernelGGL(spatial_attn32_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, (const h16*)qkv,
                       (h16*)out, N, H, nqb, (int)nb, scale * 1.4426950408889634f);
  }
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_temporal_attention(const void* qkv, void* out, int32_t B, int32_t T, int32_t S,
                                      int32_t H, int32_t D, float scale, float rope_theta, void* stream) {
  VDA_CHECK_ARG(qkv && out, "null pointer");
  VDA_CHECK_ARG(B > 0 && S > 0 && H > 0, "empty attention");
  VDA_CHECK_ARG(T > 0 && T <= 32, "temporal attention needs 1 <= T <= 32 (PE table length)");
  VDA_CHECK_ARG(D > 0 && D % 8 == 0 && D <= 128, "head dim must be a multiple of 8, <= 128");
  const long items = (long)B * S * H;
  dim3 grid((unsigned)((items + VDA_TA_NW - 1) / VDA_TA_NW));
  hipStream_t st = (hipStream_t)stream;
  const float sl = scale * 1.4426950408889634f;
  // q / k / v rows staged in LDS for the head dims the model uses (128 at C = 1024, 32 at C = 256, 8
  // heads); the direct-load kernel below serves the other head dims
  if (!g_ta_old && (D == 32 || D == 64 || D == 128)) {
    const int nw = D == 128 ? 2 : 4;  // 24 / 12 / 6 KiB of LDS per wave
    if (H % nw == 0) {
      const unsigned g = (unsigned)((items + nw - 1) / nw);
      if (D == 128)
        hipLaunchKernelGGL((temporal_attn_lds_kernel<128, 2>), dim3(g), dim3(128), 0, st, (const h16*)qkv, (h16*)out, B, T,
                           S, H, sl, rope_theta);
      else if (D == 64)
        hipLaunchKernelGGL((temporal_attn_lds_kernel<64, 4>), dim3(g), dim3(256), 0, st, (const h16*)qkv, (h16*)out, B, T,
                           S, H, sl, rope_theta);
      else
        hipLaunchKernelGGL((temporal_attn_lds_kernel<32, 4>), dim3(g), dim3(256), 0, st, (const h16*)qkv, (h16*)out, B, T,
                           S, H, sl, rope_theta);
      VDA_LAUNCH_CHECK();
      return 0;
    }
  }
  const int dp = (D + 15) / 16 * 16;
#define VDA_TA(DPV) hipLaunchKernelGGL(temporal_attn_kernel<DPV>, grid, dim3(64 * VDA_TA_NW), 0, st, (const h16*)qkv, (h16*)out, B, T, S, H, D, sl, rope_theta)
  switch (dp) {
    case 16: VDA_TA(16); break;
    case 32: VDA_TA(32); break;
    case 48: VDA_TA(48); break;
    case 64: VDA_TA(64); break;
    case 80: VDA_TA(80); break;
    case 96: VDA_TA(96); break;
    case 112: VDA_TA(112); break;
    default: VDA_TA(128); break;
  }
#undef VDA_TA
  VDA_LAUNCH_CHECK();
  return 0;
}
