// Bilinear resize, patch-embed im2col, and the C-ABI error plumbing.
#include "vda_common.h"
#include "../../include/vda.h"
#include <cstdio>
#include <cstring>

namespace {
thread_local char g_err[512] = "";
}

int vda_set_error(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "libvda error %d: %s", code, msg ? msg : "");
  return code;
}

int vda_cu_count() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {  // benign race: every thread stores the same device property
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

extern "C" const char* vda_version(void) { return "libvda 0.2 (gfx950, fp16 MFMA)"; }
extern "C" int64_t vda_epilogue_size(void) { return (int64_t)sizeof(vda_epilogue); }
extern "C" const char* vda_last_error(void) { return g_err; }

// upsample: 2 outputs per thread, non-temporal output stores.  Measured (tools/archive/bench_upsample.py,
// 2 rounds): nt stores -4 % at 148->296 / 296->518, -24 % at 74->148; 4 outputs per thread slower than 2

namespace {

// align_corners=True source coordinate (torch area_pixel_compute_source_index for bilinear)
__device__ __forceinline__ void ac_coord(int o, int in, int out, int& i0, int& i1, float& w) {
  const float sc = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  const float f = sc * (float)o;
  i0 = (int)f;
  i1 = min(i0 + 1, in - 1);
  w = ac_weight(sc, (float)o, i0);
}

// One block row per PAIR of output rows (bt, oy), (bt, oy + 1): the two source rows and the y weight
// are fixed per row, and the (ox, 8-channel chunk) index within a row needs only 32-bit math.  When
// both rows blend the same two source rows (every upscale by >= 2 pairs them), the second row reuses
// the first's four corner loads: half the L2 reads per output.  (The first version decomposed a flat
// 64-bit index per element: the 64-bit div/mod sequence held it at ~2.5 TB/s.)  Each thread writes
// UP x 16 B of each row, loads issued before any math.
template <int UP>
__global__ __launch_bounds__(256) void upsample_kernel(const h16* __restrict__ x, h16* __restrict__ y, int rows,
                                                       int H, int W, int C, int Ho, int Wo) {
  const unsigned nch = (unsigned)C >> 3;
  const unsigned row_items = (unsigned)Wo * nch;
  const float sx = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.f;
  for (int r = 2 * blockIdx.y; r < rows; r += 2 * gridDim.y) {
    const int bt = r / Ho, oy = r - bt * Ho;
    int y0, y1; float wy;
    ac_coord(oy, H, Ho, y0, y1, wy);
    const bool two = r + 1 < rows;
    const int btB = (r + 1) / Ho, oyB = r + 1 - btB * Ho;
    int y0B, y1B; float wyB;
    ac_coord(oyB, H, Ho, y0B, y1B, wyB);
    const bool share = btB == bt && y0B == y0 && y1B == y1;
    const h16* r0 = x + ((long)bt * H + y0) * W * C;
    const h16* r1 = x + ((long)bt * H + y1) * W * C;
    const h16* r0B = x + ((long)btB * H + y0B) * W * C;
    const h16* r1B = x + ((long)btB * H + y1B) * W * C;
    h16* out = y + (long)r * row_items * 8;
    h16* outB = out + (long)row_items * 8;
    const unsigned step = gridDim.x * 256u;
    for (unsigned i0 = blockIdx.x * 256u * UP + threadIdx.x; i0 < row_items; i0 += step * UP) {
      h8 a[UP], b[UP], c[UP], d[UP];
      float wx[UP];
      unsigned o0[UP], o1[UP];
#pragma unroll
      for (int u = 0; u < UP; ++u) {
        const unsigned i = min(i0 + u * 256u, row_items - 1);
        const unsigned ox = i / nch, ch = i - ox * nch;
        const float f = sx * (float)ox;
        const int x0 = (int)f, x1 = min(x0 + 1, W - 1);
        wx[u] = ac_weight(sx, (float)ox, x0);  // one explicit fma, as at every fused-resize site
        o0[u] = (unsigned)x0 * C + ch * 8;
        o1[u] = (unsigned)x1 * C + ch * 8;
        a[u] = __builtin_bit_cast(h8, ldg16(r0 + o0[u]));
        b[u] = __builtin_bit_cast(h8, ldg16(r0 + o1[u]));
        c[u] = __builtin_bit_cast(h8, ldg16(r1 + o0[u]));
        d[u] = __builtin_bit_cast(h8, ldg16(r1 + o1[u]));
      }
#pragma unroll
      for (int u = 0; u < UP; ++u) {
        const unsigned i = i0 + u * 256u;
        if (i < row_items) {
          const h8 o = bilerp8(a[u], b[u], c[u], d[u], wx[u], wy);
          __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), reinterpret_cast<u32x4*>(out + (long)i * 8));
        }
      }
      if (!two) continue;
      if (!share) {
#pragma unroll
        for (int u = 0; u < UP; ++u) {
          a[u] = __builtin_bit_cast(h8, ldg16(r0B + o0[u]));
          b[u] = __builtin_bit_cast(h8, ldg16(r0B + o1[u]));
          c[u] = __builtin_bit_cast(h8, ldg16(r1B + o0[u]));
          d[u] = __builtin_bit_cast(h8, ldg16(r1B + o1[u]));
        }
      }
#pragma unroll
      for (int u = 0; u < UP; ++u) {
        const unsigned i = i0 + u * 256u;
        if (i < row_items) {
          const h8 o = bilerp8(a[u], b[u], c[u], d[u], wx[u], wyB);
          __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), reinterpret_cast<u32x4*>(outB + (long)i * 8));
        }
      }
    }
  }
}

// A[BT*(1+np), Kp]: row 0 of each frame (cls) is zero; k = ci*196 + ky*14 + kx; zero pad k >= 588.
// Block = (up to gp patches of one patch row, patch row py, frame bt): the 3 x 14 image rows under
// those patches are read once, coalesced (8 B per lane: W and the group start are even), rounded to
// fp16 into LDS, then the group's A rows — contiguous in A — are written as 16-B chunks gathered
// from LDS.  The rounding is the same (h16)float as element-wise, so A is bit-identical.
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ img, h16* __restrict__ a, int BT, int H,
                                                     int W, int Kp, int gp) {
  extern __shared__ h16 s[];  // [ci * 14 + ky][x - x0], 42 x gp * 14
  const int pw = W / 14, np = (H / 14) * pw;
  const int py = blockIdx.y, bt = blockIdx.z, p0 = blockIdx.x * gp;
  const int ng = min(gp, pw - p0);  // patches in this block
  const int x0 = p0 * 14, srow = gp * 14;
  const int r2 = ng * 7;            // float2 per staged row
  const float* src = img + (long)bt * 3 * H * W + (long)(py * 14) * W + x0;
  constexpr int U = 8;  // loads in flight per thread (42 x 91 float2 = 15 per thread at gp = 13)
  for (int t0 = threadIdx.x; t0 < 42 * r2; t0 += 256 * U) {
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int t = t0 + j * 256, row = t / r2, c2 = t - row * r2;
      const int ci = row / 14, ky = row - ci * 14;
      if (t < 42 * r2) v[j] = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(src + ((long)ci * H + ky) * W + 2 * c2));
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int t = t0 + j * 256, row = t / r2, c2 = t - row * r2;
      typedef _Float16 h2v __attribute__((ext_vector_type(2)));
      if (t < 42 * r2) *reinterpret_cast<h2v*>(&s[row * srow + 2 * c2]) = h2v{(h16)v[j].x, (h16)v[j].y};
    }
  }
  __syncthreads();
  const int kc = Kp >> 3;
  h16* const arow = a + ((long)bt * (1 + np) + 1 + (long)py * pw + p0) * Kp;
  for (int q = threadIdx.x; q < ng * kc; q += 256) {
    const int pl = q / kc, c8 = q - pl * kc;
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = c8 * 8 + j;
      const int ci = k / 196, r = k - ci * 196, ky = r / 14, kx = r - ky * 14;
      o[j] = k < 588 ? s[(ci * 14 + ky) * srow + pl * 14 + kx] : (h16)0;
    }
    __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), reinterpret_cast<u32x4*>(arow + (long)q * 8));
  }
  if (py == 0 && blockIdx.x == 0) {  // the frame's cls row
    h16* const crow = a + (long)bt * (1 + np) * Kp;
    for (int c8 = threadIdx.x; c8 < kc; c8 += 256) stg16(crow + c8 * 8, make_uint4(0u, 0u, 0u, 0u));
  }
}

// Explicit im2col of an NHWC fp16 map for a ks x ks conv: A[m = (bt, oy, ox)][k = (ky, kx, ci)] — the
// K order of the [Cout, ks, ks, Cin] weights, so the dense GEMM on A sums the same products in the same
// order as the implicit-GEMM conv (bit-identical).  One 16-B chunk per thread; block y = output pixel.
__global__ __launch_bounds__(256) void conv_im2col_kernel(const h16* __restrict__ x, h16* __restrict__ a, int M, int H,
                                                          int W, int Cin, int Ho, int Wo, int ks, int stride, int pad) {
  const int cpt = Cin >> 3;                          // 16-B chunks per tap
  const int cpr = ks * ks * cpt;                     // per row of A
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cpr) return;
  const int tap = c / cpt, cc = c - tap * cpt;
  const int ky = tap / ks, kx = tap - ky * ks;
  for (int m = blockIdx.y; m < M; m += gridDim.y) {
    const int hw = Ho * Wo;
    const int bt = m / hw, r = m - bt * hw, oy = r / Wo, ox = r - oy * Wo;
    const int iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
      v = ldg16(x + (((long)bt * H + iy) * W + ix) * Cin + cc * 8);
    stg16(a + (long)m * cpr * 8 + c * 8, v);
  }
}

}  // namespace

// A [BT*Ho*Wo, ks*ks*Cin] for the explicit-im2col conv route (vda_gemm.hip); Cin % 8 == 0
int vda_conv_im2col(const void* x, void* a, int BT, int H, int W, int Cin, int Ho, int Wo, int ks, int stride, int pad,
                    hipStream_t st) {
  const int M = BT * Ho * Wo, cpr = ks * ks * (Cin / 8);
  hipLaunchKernelGGL(conv_im2col_kernel, dim3((unsigned)((cpr + 255) / 256), (unsigned)std::min(M, 65535)), dim3(256), 0,
                     st, (const h16*)x, (h16*)a, M, H, W, Cin, Ho, Wo, ks, stride, pad);
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_upsample_bilinear(const void* x, void* y, int32_t BT, int32_t H, int32_t W, int32_t C,
                                     int32_t Ho, int32_t Wo, void* stream) {
  VDA_CHECK_ARG(x && y, "null pointer");
  VDA_CHECK_ARG(BT > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0 && C > 0 && C % 8 == 0, "bad resize geometry");
  constexpr int UP = 2;
  const long row_items = (long)Wo * (C / 8);
  VDA_CHECK_ARG(row_items < (1L << 30) && (long)W * C < (1L << 31), "resize row too wide");
  const int gx = (int)((row_items + 256 * UP - 1) / (256 * UP));
  const int rows = BT * Ho;
  const int gy = std::min((rows + 1) / 2, 65535);
  hipLaunchKernelGGL(upsample_kernel<UP>, dim3(gx, gy), dim3(256), 0, (hipStream_t)stream, (const h16*)x, (h16*)y,
                     rows, H, W, C, Ho, Wo);
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_patch_im2col(const float* img, void* a, int32_t BT, int32_t H, int32_t W, int32_t Kp,
                                void* stream) {
  VDA_CHECK_ARG(img && a, "null pointer");
  // the LDS-staged kernel reads img in 8-byte vectors and writes A in 16-byte chunks
  VDA_CHECK_ARG((uintptr_t)img % 8 == 0 && (uintptr_t)a % 16 == 0, "img must be 8-byte and a 16-byte aligned");
  VDA_CHECK_ARG(BT > 0 && H >= 14 && W >= 14, "empty image");
  VDA_CHECK_ARG(H % 14 == 0 && W % 14 == 0, "input height/width must be multiples of the patch size 14");
  VDA_CHECK_ARG(Kp >= 588 && Kp % 8 == 0, "Kp must be >= 588 and a multiple of 8");
  VDA_CHECK_ARG(H / 14 <= 65535 && BT <= 65535, "image too tall or batch too large");
  const int pw = W / 14;
  // 13 patches per block, fewer while that leaves < 2,048 blocks (tools/ab_im2col.py over 37 .. 3:
  // 41-44 us at 32 x 518^2, 13-19 best; 3 at 2 x 70 x 518, where 13 takes 8 us)
  int gp = std::min(pw, 13);
  auto nblk = [&](int g) { return (long)BT * (H / 14) * ((pw + g - 1) / g); };
  while (gp > 3 && nblk(gp) < 2048) gp = std::max(3, (gp + 1) / 2);
  const dim3 grid((unsigned)((pw + gp - 1) / gp), (unsigned)(H / 14), (unsigned)BT);
  hipLaunchKernelGGL(im2col_kernel, grid, dim3(256), 42 * gp * 14 * 2, (hipStream_t)stream, img, (h16*)a, BT, H, W, Kp, gp);
  VDA_LAUNCH_CHECK();
  return 0;
}

