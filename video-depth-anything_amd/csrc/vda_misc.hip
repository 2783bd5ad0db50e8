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

// One block row per output row (bt, oy): the two source rows and the y weight are fixed per block,
// and the (ox, 8-channel chunk) index within a row needs only 32-bit math.  (The first version
// decomposed a flat 64-bit index per element: the 64-bit div/mod sequence held it at ~2.5 TB/s.)
// Each thread writes UP x 16 B of the row, loads issued before any math.
template <int UP>
__global__ __launch_bounds__(256) void upsample_kernel(const h16* __restrict__ x, h16* __restrict__ y, int rows,
                                                       int H, int W, int C, int Ho, int Wo) {
  const unsigned nch = (unsigned)C >> 3;
  const unsigned row_items = (unsigned)Wo * nch;
  const float sx = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.f;
  for (int r = blockIdx.y; r < rows; r += gridDim.y) {
    const int bt = r / Ho, oy = r - bt * Ho;
    int y0, y1; float wy;
    ac_coord(oy, H, Ho, y0, y1, wy);
    const h16* r0 = x + ((long)bt * H + y0) * W * C;
    const h16* r1 = x + ((long)bt * H + y1) * W * C;
    h16* out = y + (long)r * row_items * 8;
    const unsigned step = gridDim.x * 256u;
    for (unsigned i0 = blockIdx.x * 256u * UP + threadIdx.x; i0 < row_items; i0 += step * UP) {
      h8 a[UP], b[UP], c[UP], d[UP];
      float wx[UP];
#pragma unroll
      for (int u = 0; u < UP; ++u) {
        const unsigned i = min(i0 + u * 256u, row_items - 1);
        const unsigned ox = i / nch, ch = i - ox * nch;
        const float f = sx * (float)ox;
        const int x0 = (int)f, x1 = min(x0 + 1, W - 1);
        wx[u] = f - (float)x0;
        const unsigned o0 = (unsigned)x0 * C + ch * 8, o1 = (unsigned)x1 * C + ch * 8;
        a[u] = __builtin_bit_cast(h8, ldg16(r0 + o0));
        b[u] = __builtin_bit_cast(h8, ldg16(r0 + o1));
        c[u] = __builtin_bit_cast(h8, ldg16(r1 + o0));
        d[u] = __builtin_bit_cast(h8, ldg16(r1 + o1));
      }
#pragma unroll
      for (int u = 0; u < UP; ++u) {
        const unsigned i = i0 + u * 256u;
        if (i < row_items) {
          const h8 o = bilerp8(a[u], b[u], c[u], d[u], wx[u], wy);
          __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), reinterpret_cast<u32x4*>(out + (long)i * 8));
        }
      }
    }
  }
}

// A[BT*(1+np), Kp]: row 0 of each frame (cls) is zero; k = ci*196 + ky*14 + kx; zero pad k >= 588.
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ img, h16* __restrict__ a, int BT, int H,
                                                     int W, int Kp) {
  const int ph = H / 14, pw = W / 14, np = ph * pw;
  const int kc = Kp >> 3;
  const long total = (long)BT * (1 + np) * kc;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c8 = (int)(i % kc);
    const long row = i / kc;
    const int tok = (int)(row % (1 + np));
    const int bt = (int)(row / (1 + np));
    h8 o;
    if (tok == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (h16)0;
    } else {
      const int p = tok - 1, py = p / pw, px = p - py * pw;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = c8 * 8 + j;
        float v = 0.f;
        if (k < 588) {
          const int ci = k / 196, r = k - ci * 196, ky = r / 14, kx = r - ky * 14;
          v = img[(((long)bt * 3 + ci) * H + py * 14 + ky) * W + px * 14 + kx];
        }
        o[j] = (h16)v;
      }
    }
    stg16(a + i * 8, __builtin_bit_cast(uint4, o));
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
  const int gy = std::min(rows, 65535);
  hipLaunchKernelGGL(upsample_kernel<UP>, dim3(gx, gy), dim3(256), 0, (hipStream_t)stream, (const h16*)x, (h16*)y,
                     rows, H, W, C, Ho, Wo);
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_patch_im2col(const float* img, void* a, int32_t BT, int32_t H, int32_t W, int32_t Kp,
                                void* stream) {
  VDA_CHECK_ARG(img && a, "null pointer");
  VDA_CHECK_ARG(BT > 0 && H >= 14 && W >= 14, "empty image");
  VDA_CHECK_ARG(H % 14 == 0 && W % 14 == 0, "input height/width must be multiples of the patch size 14");
  VDA_CHECK_ARG(Kp >= 588 && Kp % 8 == 0, "Kp must be >= 588 and a multiple of 8");
  const long total = (long)BT * (1 + (H / 14) * (W / 14)) * (Kp / 8);
  const int grid = (int)std::min<long>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(im2col_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, img, (h16*)a, BT, H, W, Kp);
  VDA_LAUNCH_CHECK();
  return 0;
}

