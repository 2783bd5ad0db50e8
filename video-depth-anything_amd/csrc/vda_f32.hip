// fp32 mode of the clip forward (infer_video_depth(fp32=True), video_depth.py:366-368 with
// autocast off): every op in fp32 storage with fp32 accumulation, so the result tracks the
// reference's fp32 path to summation-order rounding (parity tier (i)).
//
// Contractions run on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32: f32 in, f32 accumulate, no
// xf32 on gfx950), 157 TF/s peak.  Same data layout as the fp16 path (token-major / NHWC, weights
// K-contiguous), same epilogue contract (include/vda.h vda_epilogue, residuals as float).
//
//   gemm_f32_kernel     128x128 tile, 4 waves (2 m x 2 n, wave tile 64x64), BK = 16, register-
//                       staged double-buffered LDS with rows padded to 20 floats (conflict-free
//                       16-lane fragment reads, 16-B aligned stores).  A = W (lane owns 4
//                       consecutive output channels), B = X.  Dense or implicit-GEMM conv loader.
//   spatial_attn_f32    flash attention, 64 queries per block (16 per wave), 64-key K/V blocks in
//                       LDS; S^T = K Q^T and O^T = V^T P^T on the f32 MFMA, online softmax in fp32
//                       with expf; P feeds the PV product from the S accumulator registers (the
//                       key order of a k-step is permuted identically on both operands).
//   temporal_attn_f32   one wave per (site, head), lane = query frame (T <= 32), K/V/Q^T in LDS.
//   layernorm / groupnorm / upsample / im2col / depth tail: fp32 versions of the fp16 kernels.
#include "vda_common.h"
#include "../../include/vda.h"
#include <cmath>

namespace {

struct F32Params {
  const float* x; long ldx;
  const float* w;
  float* y; long ldy;
  int M, N, K;
  int H, W, Cin, Ho, Wo, ks, stride, pad, pre_relu;
  vda_epilogue epi;
};

constexpr int FBK = 16;   // K per LDS tile
constexpr int FLD = 20;   // padded LDS row (floats)

__device__ __forceinline__ f4 mfma_f32(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float gelu_exact(float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); }

template <bool CONV>
__device__ __forceinline__ f4 load_x4(const F32Params& p, int m, int k, int bt, int oy, int ox) {
  if (m >= p.M || k >= p.K) return f4{0.f, 0.f, 0.f, 0.f};
  if constexpr (CONV) {
    const int tap = k / p.Cin, ci = k - tap * p.Cin;
    const int ky = tap / p.ks, kx = tap - ky * p.ks;
    const int iy = oy * p.stride - p.pad + ky, ix = ox * p.stride - p.pad + kx;
    if (iy < 0 || iy >= p.H || ix < 0 || ix >= p.W) return f4{0.f, 0.f, 0.f, 0.f};
    f4 v = *reinterpret_cast<const f4*>(p.x + (((long)bt * p.H + iy) * p.W + ix) * p.Cin + ci);
    if (p.pre_relu) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    return v;
  } else {
    return *reinterpret_cast<const f4*>(p.x + (long)m * p.ldx + k);
  }
}

template <int ACT>
__device__ __forceinline__ void epi_f32(const F32Params& p, int m, int n, f4 v) {
  const vda_epilogue& e = p.epi;
  if (e.bias) v += *reinterpret_cast<const f4*>(e.bias + n);
  if (e.rowbias) v += *reinterpret_cast<const f4*>(e.rowbias + (long)((m / e.rdiv) % e.rmod) * p.N + n);
  if constexpr (ACT == VDA_ACT_GELU) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = gelu_exact(v[j]);
  } else if constexpr (ACT == VDA_ACT_RELU) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
  }
  if (e.gamma) v *= *reinterpret_cast<const f4*>(e.gamma + n);
  if (e.res) v += *reinterpret_cast<const f4*>((const float*)e.res + (long)m * e.ldres + n);
  if (e.res2) v += *reinterpret_cast<const f4*>((const float*)e.res2 + (long)m * e.ldres2 + n);
  long off;
  if (e.store == VDA_STORE_PIXEL_SHUFFLE) {
    const int k = e.ps_k, cout = e.ps_cout;
    const int ij = n / cout, co = n - ij * cout;
    const int ki = ij / k, kj = ij - ki * k;
    const int xw = m % e.ps_win;
    const int t = m / e.ps_win;
    const int yh = t % e.ps_hin, bt = t / e.ps_hin;
    off = (((long)bt * e.ps_hin * k + (long)yh * k + ki) * ((long)e.ps_win * k) + (long)xw * k + kj) * cout + co;
  } else {
    off = (long)m * p.ldy + n;
  }
  *reinterpret_cast<f4*>(p.y + off) = v;
}

template <bool CONV, int ACT>
__global__ __launch_bounds__(256) void gemm_f32_kernel(F32Params p, int tiles_n) {
  __shared__ float xs[2][128 * FLD];
  __shared__ float ws[2][128 * FLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int tn = blockIdx.x % tiles_n, tm = blockIdx.x / tiles_n;
  const int m0 = tm * 128, n0 = tn * 128;
  // global -> register staging: rows r = tid>>2 (+64), 4-float chunk c = tid&3
  const int lr = tid >> 2, lc = (tid & 3) * 4;
  int bt[2] = {0, 0}, oy[2] = {0, 0}, ox[2] = {0, 0};
  if constexpr (CONV) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = min(m0 + lr + 64 * i, p.M - 1);
      ox[i] = m % p.Wo;
      const int t = m / p.Wo;
      oy[i] = t % p.Ho;
      bt[i] = t / p.Ho;
    }
  }
  f4 rx[2], rw[2];
  auto gload = [&](int kt) {
    const int k = kt * FBK + lc;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      rx[i] = load_x4<CONV>(p, m0 + lr + 64 * i, k, bt[i], oy[i], ox[i]);
      const int n = n0 + lr + 64 * i;
      rw[i] = (n < p.N && k < p.K) ? *reinterpret_cast<const f4*>(p.w + (long)n * p.K + k) : f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<f4*>(&xs[buf][(lr + 64 * i) * FLD + lc]) = rx[i];
      *reinterpret_cast<f4*>(&ws[buf][(lr + 64 * i) * FLD + lc]) = rw[i];
    }
  };
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int nk = (p.K + FBK - 1) / FBK;
  gload(0);
  sstore(0);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cb = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
#pragma unroll
    for (int kk = 0; kk < FBK / 4; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = ws[cb][(wn * 64 + i * 16 + fr) * FLD + kk * 4 + fk];
        b[i] = xs[cb][(wm * 64 + i * 16 + fr) * FLD + kk * 4 + fk];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma_f32(a[i], b[j], acc[i][j]);
    }
    if (kt + 1 < nk) sstore(cb ^ 1);
    __syncthreads();
  }
  // C/D: row (n) = (lane >> 4) * 4 + r, col (m) = lane & 15
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + wm * 64 + j * 16 + fr;
    if (m >= p.M) continue;
    if constexpr (ACT == VDA_ACT_GEGLU) {
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int nb = n0 + wn * 64 + pr * 32;  // 32-row [h16 | g16] block
        const int nh = nb + fk * 4, ng = nh + 16, nout = nb / 2 + fk * 4;
        if (nh >= p.N) continue;
        f4 vh = acc[2 * pr][j], vg = acc[2 * pr + 1][j];
        const vda_epilogue& e = p.epi;
        if (e.bias) {
          vh += *reinterpret_cast<const f4*>(e.bias + nh);
          vg += *reinterpret_cast<const f4*>(e.bias + ng);
        }
        f4 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = vh[q] * gelu_exact(vg[q]);
        if (e.gamma) v *= *reinterpret_cast<const f4*>(e.gamma + nout);
        if (e.res) v += *reinterpret_cast<const f4*>((const float*)e.res + (long)m * e.ldres + nout);
        *reinterpret_cast<f4*>(p.y + (long)m * p.ldy + nout) = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = n0 + wn * 64 + i * 16 + fk * 4;
        if (n < p.N) epi_f32<ACT>(p, m, n, acc[i][j]);
      }
    }
  }
}

// ---- spatial attention (fp32 flash) -----------------------------------------------------------
constexpr int SLD = 68;  // padded K/V LDS row (floats): conflict-free fragment reads

__global__ __launch_bounds__(256) void spatial_attn_f32_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                               int N, int H, float scale) {
  constexpr int D = 64;
  __shared__ float ks[64 * SLD];
  __shared__ float vs[64 * SLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = blockIdx.y, b = blockIdx.z;
  const int q0 = blockIdx.x * 64 + wave * 16;
  const long ld = 3L * H * D;
  const float* base = qkv + (long)b * N * ld;
  const int fr = lane & 15, fk = lane >> 4;
  // Q^T fragments (B operand): lane holds Q[q0 + fr][4 s + fk] * scale, s = 0..15
  float qf[16];
  {
    const int q = min(q0 + fr, N - 1);
    const float* qr = base + (long)q * ld + h * D;
#pragma unroll
    for (int s = 0; s < 16; ++s) qf[s] = qr[4 * s + fk] * scale;
  }
  f4 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f4{0.f, 0.f, 0.f, 0.f};
  float mrun = -INFINITY, lrun = 0.f;
  const int nkb = (N + 63) / 64;
  for (int kb = 0; kb < nkb; ++kb) {
    __syncthreads();
    // stage K and V rows kb*64 .. +63 (zeros past N)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i;         // 1024 float4 per operand
      const int r = idx >> 4, c = (idx & 15) * 4;
      const int key = kb * 64 + r;
      f4 kv = f4{0.f, 0.f, 0.f, 0.f}, vv = f4{0.f, 0.f, 0.f, 0.f};
      if (key < N) {
        const float* row = base + (long)key * ld;
        kv = *reinterpret_cast<const f4*>(row + (H + h) * D + c);
        vv = *reinterpret_cast<const f4*>(row + (2 * H + h) * D + c);
      }
      *reinterpret_cast<f4*>(&ks[r * SLD + c]) = kv;
      *reinterpret_cast<f4*>(&vs[r * SLD + c]) = vv;
    }
    __syncthreads();
    // S^T[key][q] for 4 key sub-blocks: lane holds keys kbs*16 + fk*4 + r of query fr
    f4 s4[4];
#pragma unroll
    for (int kbs = 0; kbs < 4; ++kbs) {
      f4 a = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 16; ++s) a = mfma_f32(ks[(kbs * 16 + fr) * SLD + 4 * s + fk], qf[s], a);
      s4[kbs] = a;
    }
    float bmax = -INFINITY;
#pragma unroll
    for (int kbs = 0; kbs < 4; ++kbs)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kb * 64 + kbs * 16 + fk * 4 + r;
        if (key >= N) s4[kbs][r] = -INFINITY;
        bmax = fmaxf(bmax, s4[kbs][r]);
      }
    bmax = fmaxf(bmax, __shfl_xor(bmax, 16, 64));
    bmax = fmaxf(bmax, __shfl_xor(bmax, 32, 64));
    const float mnew = fmaxf(mrun, bmax);
    const float corr = expf(mrun - mnew);
    float psum = 0.f;
#pragma unroll
    for (int kbs = 0; kbs < 4; ++kbs)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = expf(s4[kbs][r] - mnew);
        s4[kbs][r] = pv;
        psum += pv;
      }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    lrun = lrun * corr + psum;
    mrun = mnew;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] *= corr;
    // O^T[d][q] += sum_key V[key][d] P[q][key]; k-step (kbs, r): lane supplies key kbs*16 + fk*4 + r
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int kbs = 0; kbs < 4; ++kbs)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          o[db] = mfma_f32(vs[(kbs * 16 + fk * 4 + r) * SLD + db * 16 + fr], s4[kbs][r], o[db]);
  }
  // o[db][rr] = O[q = fr][d = db*16 + fk*4 + rr]
  const int q = q0 + fr;
  if (q < N) {
    const float inv = 1.f / lrun;
    float* orow = out + ((long)b * N + q) * H * D + h * D;
#pragma unroll
    for (int db = 0; db < 4; ++db) *reinterpret_cast<f4*>(orow + db * 16 + fk * 4) = o[db] * inv;
  }
}

// ---- temporal attention (fp32) ----------------------------------------------------------------
// One wave per (b, site, head); lane t < T is query frame t.  qkv rows (b*T + t)*S + s.
__global__ __launch_bounds__(64) void temporal_attn_f32_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                               int T, int S, int H, int D, float scale,
                                                               float rope_theta) {
  __shared__ float qt[128 * 33];  // Q^T [d][t] (row 33 floats)
  __shared__ float kk[32 * 129];  // K [t][d]
  __shared__ float vv[32 * 129];  // V [t][d]
  const int lane = threadIdx.x;
  const int h = blockIdx.x % H;
  const int site = blockIdx.x / H;  // b * S + s
  const int b = site / S, s = site - b * S;
  const int C = H * D;
  const long ld = 3L * C;
  // channel pairs (d, d+1): pe='rope' rotates q and k by t * theta^(-2i/C), i = global pair index
  // (attention.py:403-429); D is even for every head size (D % 8 == 0 is not required here)
  const int Dh = D >> 1;
  for (int i = lane; i < T * Dh; i += 64) {
    const int t = i / Dh, d = 2 * (i - t * Dh);
    const float* row = qkv + ((long)(b * T + t) * S + s) * ld + h * D + d;
    float qa = row[0], qb = row[1], ka = row[C], kb = row[C + 1];
    if (rope_theta > 0.f) {
      const int pi = (h * D + d) >> 1;
      const float freq = 1.f / powf(rope_theta, (float)(2 * pi) / (float)C);
      float sn, cs;
      sincosf((float)t * freq, &sn, &cs);
      const float q0 = qa * cs - qb * sn, q1 = qa * sn + qb * cs;
      const float k0 = ka * cs - kb * sn, k1 = ka * sn + kb * cs;
      qa = q0; qb = q1; ka = k0; kb = k1;
    }
    qt[d * 33 + t] = qa;
    qt[(d + 1) * 33 + t] = qb;
    kk[t * 129 + d] = ka;
    kk[t * 129 + d + 1] = kb;
    vv[t * 129 + d] = row[2 * C];
    vv[t * 129 + d + 1] = row[2 * C + 1];
  }
  __syncthreads();
  if (lane >= T) return;
  float sc[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) sc[j] = 0.f;
  for (int d = 0; d < D; ++d) {
    const float qd = qt[d * 33 + lane];
#pragma unroll
    for (int j = 0; j < 32; ++j)
      if (j < T) sc[j] = fmaf(qd, kk[j * 129 + d], sc[j]);
  }
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < 32; ++j)
    if (j < T) { sc[j] *= scale; mx = fmaxf(mx, sc[j]); }
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 32; ++j)
    if (j < T) { sc[j] = expf(sc[j] - mx); sum += sc[j]; }
  const float inv = 1.f / sum;
#pragma unroll
  for (int j = 0; j < 32; ++j) sc[j] *= inv;
  float* orow = out + ((long)(b * T + lane) * S + s) * C + h * D;
  for (int d = 0; d < D; ++d) {
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j)
      if (j < T) a = fmaf(sc[j], vv[j * 129 + d], a);
    orow[d] = a;
  }
}

// ---- norms, resize, im2col, depth tail --------------------------------------------------------
// One wave per row, C <= 2048 (32 floats per lane), two-pass statistics.
__global__ __launch_bounds__(256) void layernorm_f32_kernel(const float* __restrict__ x, long ldx, float* __restrict__ y,
                                                            const float* __restrict__ g, const float* __restrict__ bb,
                                                            int rows, int C, float eps, int skip_period) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const long src = skip_period > 0 ? (long)row + row / skip_period + 1 : (long)row;
  const float* xr = x + src * ldx;
  float v[32];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < C ? xr[c] : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int c = lane + 64 * i;
    if (c < C) { const float d = v[i] - mean; q += d * d; }
  }
  const float rstd = 1.f / sqrtf(wave_sum(q) / (float)C + eps);
  float* yr = y + (long)row * C;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int c = lane + 64 * i;
    if (c < C) yr[c] = (v[i] - mean) * rstd * g[c] + bb[c];
  }
}

__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// One block per (frame, group): slab of S rows x cg channels at row stride C.
__global__ __launch_bounds__(256) void groupnorm_f32_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                            const float* __restrict__ g, const float* __restrict__ bb,
                                                            int S, int C, int groups, float eps) {
  __shared__ float red[4];
  const int f = blockIdx.x / groups, grp = blockIdx.x % groups;
  const int cg = C / groups;
  const long n = (long)S * cg;
  const float* base = x + (long)f * S * C + grp * cg;
  float* ob = y + (long)f * S * C + grp * cg;
  float s = 0.f;
  for (long i = threadIdx.x; i < n; i += 256) s += base[(i / cg) * C + i % cg];
  const float mean = block_sum256(s, red) / (float)n;
  float q = 0.f;
  for (long i = threadIdx.x; i < n; i += 256) { const float d = base[(i / cg) * C + i % cg] - mean; q += d * d; }
  const float rstd = 1.f / sqrtf(block_sum256(q, red) / (float)n + eps);
  for (long i = threadIdx.x; i < n; i += 256) {
    const int c = (int)(i % cg);
    const long off = (i / cg) * C + c;
    ob[off] = (base[off] - mean) * rstd * g[grp * cg + c] + bb[grp * cg + c];
  }
}

// bilinear align_corners=True, NHWC, 4 channels per thread (torch upsample_bilinear2d weights)
__global__ __launch_bounds__(256) void upsample_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int BT,
                                                           int H, int W, int C, int Ho, int Wo) {
  const int nc = C >> 2;
  const long total = (long)BT * Ho * Wo * nc;
  const float ry = Ho > 1 ? (float)(H - 1) / (float)(Ho - 1) : 0.f;
  const float rx = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % nc);
    long t = i / nc;
    const int ox = (int)(t % Wo); t /= Wo;
    const int oy = (int)(t % Ho);
    const int bt = (int)(t / Ho);
    const float sy = ry * (float)oy, sx = rx * (float)ox;
    const int y0 = (int)sy, x0 = (int)sx;
    const int y1 = y0 + (y0 < H - 1), x1 = x0 + (x0 < W - 1);
    const float ly = sy - (float)y0, lx = sx - (float)x0;
    const float hy = 1.f - ly, hx = 1.f - lx;
    const float* bp = x + (long)bt * H * W * C + c * 4;
    const f4 a = *reinterpret_cast<const f4*>(bp + ((long)y0 * W + x0) * C);
    const f4 bq = *reinterpret_cast<const f4*>(bp + ((long)y0 * W + x1) * C);
    const f4 cq = *reinterpret_cast<const f4*>(bp + ((long)y1 * W + x0) * C);
    const f4 d = *reinterpret_cast<const f4*>(bp + ((long)y1 * W + x1) * C);
    f4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = hy * (hx * a[j] + lx * bq[j]) + ly * (hx * cq[j] + lx * d[j]);
    *reinterpret_cast<f4*>(y + i * 4) = o;
  }
}

__global__ __launch_bounds__(256) void im2col_f32_kernel(const float* __restrict__ img, float* __restrict__ a, int BT,
                                                         int H, int W, int Kp) {
  const int ph = H / 14, pw = W / 14, np = ph * pw;
  const long total = (long)BT * (1 + np) * Kp;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int k = (int)(i % Kp);
    const long row = i / Kp;
    const int tok = (int)(row % (1 + np));
    const int bt = (int)(row / (1 + np));
    float v = 0.f;
    if (tok > 0 && k < 588) {
      const int pidx = tok - 1, py = pidx / pw, px = pidx - py * pw;
      const int ci = k / 196, r = k - ci * 196, ky = r / 14, kx = r - ky * 14;
      v = img[(((long)bt * 3 + ci) * H + py * 14 + ky) * W + px * 14 + kx];
    }
    a[i] = v;
  }
}

// depth = relu(sum_c mid[m, c] * w2[c] + b2), mid [M, 32] (already ReLU'd by the conv epilogue)
__global__ __launch_bounds__(256) void pointwise_relu_f32_kernel(const float* __restrict__ mid, const float* __restrict__ w2,
                                                                 const float* __restrict__ b2, float* __restrict__ out, long M) {
  const long m = (long)blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  const float* r = mid + m * 32;
  float a = 0.f;
#pragma unroll
  for (int c = 0; c < 32; c += 4) {
    const f4 v = *reinterpret_cast<const f4*>(r + c);
    a += v[0] * w2[c] + v[1] * w2[c + 1] + v[2] * w2[c + 2] + v[3] * w2[c + 3];
  }
  out[m] = fmaxf(a + b2[0], 0.f);
}

template <bool CONV>
int launch_f32(const F32Params& p, hipStream_t st) {
  const int tiles_n = (p.N + 127) / 128, tiles_m = (p.M + 127) / 128;
  const long blocks = (long)tiles_n * tiles_m;
  if (blocks > 0x7fffffffL) return vda_set_error(-22, "fp32 GEMM grid too large");
  const dim3 g((unsigned)blocks), bl(256);
  switch (p.epi.act) {
    case VDA_ACT_NONE: hipLaunchKernelGGL((gemm_f32_kernel<CONV, VDA_ACT_NONE>), g, bl, 0, st, p, tiles_n); break;
    case VDA_ACT_GELU: hipLaunchKernelGGL((gemm_f32_kernel<CONV, VDA_ACT_GELU>), g, bl, 0, st, p, tiles_n); break;
    case VDA_ACT_RELU: hipLaunchKernelGGL((gemm_f32_kernel<CONV, VDA_ACT_RELU>), g, bl, 0, st, p, tiles_n); break;
    case VDA_ACT_GEGLU:
      if (CONV) return vda_set_error(-22, "GEGLU epilogue is dense-only");
      hipLaunchKernelGGL((gemm_f32_kernel<CONV, VDA_ACT_GEGLU>), g, bl, 0, st, p, tiles_n);
      break;
    default: return vda_set_error(-22, "unknown activation");
  }
  VDA_LAUNCH_CHECK();
  return 0;
}

}  // namespace

extern "C" int vda_gemm_f32(const float* x, int64_t ldx, const float* w, float* y, int64_t ldy, int32_t M, int32_t N,
                            int32_t K, const vda_epilogue* epi, void* stream) {
  VDA_CHECK_ARG(x && w && y && epi, "null pointer");
  VDA_CHECK_ARG(M > 0 && N > 0 && K > 0, "empty GEMM");
  VDA_CHECK_ARG(K % 4 == 0 && ldx % 4 == 0 && N % 4 == 0, "fp32 GEMM needs K, ldx, N multiples of 4");
  VDA_CHECK_ARG(epi->act != VDA_ACT_GEGLU || N % 32 == 0, "GEGLU needs N % 32 == 0");
  VDA_CHECK_ARG(epi->store != VDA_STORE_PIXEL_SHUFFLE || (epi->ps_k > 0 && epi->ps_cout % 4 == 0 &&
                                                         epi->ps_hin > 0 && epi->ps_win > 0),
                "bad pixel-shuffle geometry");
  VDA_CHECK_ARG(!epi->rowbias || (epi->rdiv > 0 && epi->rmod > 0), "rowbias needs rdiv, rmod > 0");
  VDA_CHECK_ARG(!epi->ln_stats, "fp32 GEMM: no LayerNorm fold (the fp32 mode runs vda_layernorm_f32)");
  VDA_CHECK_ARG(!epi->stats_out, "fp32 GEMM: no row statistics output");
  VDA_CHECK_ARG(epi->res2_h == 0 && epi->res2_w == 0, "fp32 GEMM: no upsampled res2");
  F32Params p{};
  p.x = x; p.ldx = ldx; p.w = w; p.y = y; p.ldy = ldy; p.M = M; p.N = N; p.K = K; p.epi = *epi;
  return launch_f32<false>(p, (hipStream_t)stream);
}

extern "C" int vda_conv2d_f32(const float* x, const float* w, float* y, int32_t BT, int32_t H, int32_t W, int32_t Cin,
                              int32_t Cout, int32_t ks, int32_t stride, int32_t pad, int32_t pre_relu,
                              const vda_epilogue* epi, void* stream) {
  VDA_CHECK_ARG(x && w && y && epi, "null pointer");
  VDA_CHECK_ARG(BT > 0 && H > 0 && W > 0 && ks > 0 && stride > 0 && pad >= 0, "bad conv geometry");
  VDA_CHECK_ARG(Cin % 4 == 0 && Cout % 4 == 0, "fp32 conv needs Cin, Cout multiples of 4");
  VDA_CHECK_ARG(epi->act != VDA_ACT_GEGLU && epi->store == VDA_STORE_ROWS, "conv epilogue: no GEGLU / pixel shuffle");
  VDA_CHECK_ARG(epi->res2_h == 0 && epi->res2_w == 0, "fp32 conv: no upsampled res2 (materialise it)");
  F32Params p{};
  p.x = x; p.w = w; p.y = y; p.ldy = Cout;
  p.H = H; p.W = W; p.Cin = Cin; p.ks = ks; p.stride = stride; p.pad = pad; p.pre_relu = pre_relu;
  p.Ho = (H + 2 * pad - ks) / stride + 1;
  p.Wo = (W + 2 * pad - ks) / stride + 1;
  VDA_CHECK_ARG(p.Ho > 0 && p.Wo > 0, "empty conv output");
  const long M = (long)BT * p.Ho * p.Wo;
  VDA_CHECK_ARG(M < 0x7fffffffL, "conv output too large");
  p.M = (int)M; p.N = Cout; p.K = ks * ks * Cin; p.epi = *epi;
  return launch_f32<true>(p, (hipStream_t)stream);
}

extern "C" int vda_spatial_attention_f32(const float* qkv, float* out, int32_t B, int32_t N, int32_t H, int32_t D,
                                         float scale, void* stream) {
  VDA_CHECK_ARG(qkv && out, "null pointer");
  VDA_CHECK_ARG(B > 0 && N > 0 && H > 0, "empty attention");
  VDA_CHECK_ARG(D == 64, "fp32 spatial attention: head dim must be 64");
  VDA_CHECK_ARG(B <= 65535 && H <= 65535, "grid too large");
  hipLaunchKernelGGL(spatial_attn_f32_kernel, dim3((N + 63) / 64, H, B), dim3(256), 0, (hipStream_t)stream, qkv, out, N,
                     H, scale);
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_temporal_attention_f32(const float* qkv, float* out, int32_t B, int32_t T, int32_t S, int32_t H,
                                          int32_t D, float scale, float rope_theta, void* stream) {
  VDA_CHECK_ARG(qkv && out, "null pointer");
  VDA_CHECK_ARG(B > 0 && T > 0 && S > 0 && H > 0 && D > 0, "empty attention");
  VDA_CHECK_ARG(T <= 32 && D <= 128 && D % 2 == 0, "temporal attention: T <= 32, even D <= 128");
  const long blocks = (long)B * S * H;
  VDA_CHECK_ARG(blocks < 0x7fffffffL, "grid too large");
  hipLaunchKernelGGL(temporal_attn_f32_kernel, dim3((unsigned)blocks), dim3(64), 0, (hipStream_t)stream, qkv, out, T, S,
                     H, D, scale, rope_theta);
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_layernorm_f32(const float* x, int64_t ldx, float* y, const float* gamma, const float* beta,
                                 int32_t rows, int32_t C, float eps, int32_t skip_period, void* stream) {
  VDA_CHECK_ARG(x && y && gamma && beta, "null pointer");
  VDA_CHECK_ARG(rows > 0 && C > 0 && C <= 2048, "LayerNorm: 0 < C <= 2048");
  hipLaunchKernelGGL(layernorm_f32_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, x, (long)ldx, y,
                     gamma, beta, rows, C, eps, skip_period);
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_groupnorm_f32(const float* x, float* y, const float* gamma, const float* beta, int32_t F, int32_t S,
                                 int32_t C, int32_t groups, float eps, void* stream) {
  VDA_CHECK_ARG(x && y && gamma && beta, "null pointer");
  VDA_CHECK_ARG(F > 0 && S > 0 && groups > 0 && C % groups == 0, "bad GroupNorm geometry");
  hipLaunchKernelGGL(groupnorm_f32_kernel, dim3(F * groups), dim3(256), 0, (hipStream_t)stream, x, y, gamma, beta, S, C,
                     groups, eps);
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_upsample_bilinear_f32(const float* x, float* y, int32_t BT, int32_t H, int32_t W, int32_t C,
                                         int32_t Ho, int32_t Wo, void* stream) {
  VDA_CHECK_ARG(x && y, "null pointer");
  VDA_CHECK_ARG(BT > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0 && C > 0 && C % 4 == 0, "bad resize geometry");
  const long total = (long)BT * Ho * Wo * (C / 4);
  const int grid = (int)std::min<long>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(upsample_f32_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, y, BT, H, W, C, Ho, Wo);
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_patch_im2col_f32(const float* img, float* a, int32_t BT, int32_t H, int32_t W, int32_t Kp,
                                    void* stream) {
  VDA_CHECK_ARG(img && a, "null pointer");
  VDA_CHECK_ARG(BT > 0 && H >= 14 && W >= 14 && H % 14 == 0 && W % 14 == 0, "bad image geometry");
  VDA_CHECK_ARG(Kp >= 588 && Kp % 4 == 0, "Kp must be >= 588 and a multiple of 4");
  const long total = (long)BT * (1 + (H / 14) * (W / 14)) * Kp;
  const int grid = (int)std::min<long>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(im2col_f32_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, img, a, BT, H, W, Kp);
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_depth_head_f32(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                                  float* depth, float* ws_up, float* ws_mid, int32_t BT, int32_t Hin, int32_t Win,
                                  int32_t C, int32_t Ho, int32_t Wo, void* stream) {
  VDA_CHECK_ARG(x && w1 && b1 && w2 && b2 && depth && ws_up && ws_mid, "null pointer");
  int rc = vda_upsample_bilinear_f32(x, ws_up, BT, Hin, Win, C, Ho, Wo, stream);
  if (rc) return rc;
  vda_epilogue e{};
  e.bias = b1;
  e.rdiv = e.rmod = 1;
  e.act = VDA_ACT_RELU;
  rc = vda_conv2d_f32(ws_up, w1, ws_mid, BT, Ho, Wo, C, 32, 3, 1, 1, 0, &e, stream);
  if (rc) return rc;
  const long M = (long)BT * Ho * Wo;
  hipLaunchKernelGGL(pointwise_relu_f32_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     ws_mid, w2, b2, depth, M);
  VDA_LAUNCH_CHECK();
  return 0;
}
