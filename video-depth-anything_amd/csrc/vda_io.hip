// Frame preprocessing and depth post-resize: the data formats either side of the clip forward.
//
// preprocess: uint8 RGB frames [N, h, w, 3] (HWC, as decoded video frames arrive) -> the network
// input [N, 3, H, W] float: x / 255, bicubic resize (a = -0.75, half-pixel centres, clamped
// borders, no antialias: cv2.INTER_CUBIC == torch bicubic align_corners=False), then
// (x - mean) / std.  Replaces util/transform.py:5-157 (Resize + NormalizeImage + PrepareForNet)
// as applied per frame in video_depth.py:336-361 / :140-146 / :209.
//
// depth_resize: depth [N, H, W] float -> [N, ho, wo] float, bilinear align_corners=True
// (video_depth.py:372, :300).
//
// Both are HBM/latency-bound elementwise gathers: one thread per output pixel, consecutive
// threads on consecutive output columns so every store is a coalesced row segment; the 4x4 (or
// 2x2) source window of neighbouring threads overlaps and is served from L1/L2.
#include "vda_common.h"
#include "../../include/vda.h"

namespace {

constexpr float kCubicA = -0.75f;

// torch upsample_bicubic2d / cv2 INTER_CUBIC kernel weights for fractional offset t
__device__ __forceinline__ void cubic_weights(float t, float w[4]) {
  const float A = kCubicA;
  const float x0 = t + 1.f;   // |x| in (1, 2)
  const float x1 = t;         // |x| in [0, 1]
  const float x2 = 1.f - t;   // |x| in [0, 1]
  const float x3 = 2.f - t;   // |x| in (1, 2)
  w[0] = ((A * x0 - 5.f * A) * x0 + 8.f * A) * x0 - 4.f * A;
  w[1] = ((A + 2.f) * x1 - (A + 3.f)) * x1 * x1 + 1.f;
  w[2] = ((A + 2.f) * x2 - (A + 3.f)) * x2 * x2 + 1.f;
  w[3] = ((A * x3 - 5.f * A) * x3 + 8.f * A) * x3 - 4.f * A;
}

struct NormArgs {
  float mean[3];
  float std_[3];
};

__global__ __launch_bounds__(256) void preprocess_kernel(const uint8_t* __restrict__ src, float* __restrict__ dst,
                                                         int h, int w, int H, int W, NormArgs na) {
  const int ox = blockIdx.x * 256 + threadIdx.x;
  const int oy = blockIdx.y;
  const int n = blockIdx.z;
  if (ox >= W) return;
  // half-pixel source coordinates, not clamped (cubic), floor + fraction (torch
  // area_pixel_compute_source_index(cubic=true))
  const float sy = (float)h / (float)H * ((float)oy + 0.5f) - 0.5f;
  const float sx = (float)w / (float)W * ((float)ox + 0.5f) - 0.5f;
  const float fy = floorf(sy), fx = floorf(sx);
  const int iy = (int)fy, ix = (int)fx;
  float wy[4], wx[4];
  cubic_weights(sy - fy, wy);
  cubic_weights(sx - fx, wx);
  int cols[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) cols[k] = min(max(ix - 1 + k, 0), w - 1) * 3;
  const uint8_t* frame = src + (size_t)n * h * w * 3;
  float acc[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint8_t* row = frame + (size_t)min(max(iy - 1 + r, 0), h - 1) * w * 3;
    float rv[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int c = 0; c < 3; ++c) rv[c] += (float)row[cols[k] + c] / 255.f * wx[k];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) acc[c] += rv[c] * wy[r];
  }
  const size_t plane = (size_t)H * W;
  float* out = dst + (size_t)n * 3 * plane + (size_t)oy * W + ox;
#pragma unroll
  for (int c = 0; c < 3; ++c) out[c * plane] = (acc[c] - na.mean[c]) / na.std_[c];
}

__global__ __launch_bounds__(256) void depth_resize_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                           int H, int W, int ho, int wo) {
  const int ox = blockIdx.x * 256 + threadIdx.x;
  const int oy = blockIdx.y;
  const int n = blockIdx.z;
  if (ox >= wo) return;
  // align_corners=True: src = o * (in - 1) / (out - 1)  (torch upsample_bilinear2d)
  const float ry = ho > 1 ? (float)(H - 1) / (float)(ho - 1) : 0.f;
  const float rx = wo > 1 ? (float)(W - 1) / (float)(wo - 1) : 0.f;
  const float sy = ry * (float)oy, sx = rx * (float)ox;
  const int y0 = (int)sy, x0 = (int)sx;
  const int y1 = y0 + (y0 < H - 1 ? 1 : 0), x1 = x0 + (x0 < W - 1 ? 1 : 0);
  const float ly = sy - (float)y0, lx = sx - (float)x0;
  const float* f = src + (size_t)n * H * W;
  const float v = (1.f - ly) * ((1.f - lx) * f[(size_t)y0 * W + x0] + lx * f[(size_t)y0 * W + x1]) +
                  ly * ((1.f - lx) * f[(size_t)y1 * W + x0] + lx * f[(size_t)y1 * W + x1]);
  dst[((size_t)n * ho + oy) * wo + ox] = v;
}

}  // namespace

extern "C" int vda_preprocess_frames(const void* frames, float* out, int32_t N, int32_t h, int32_t w, int32_t H,
                                     int32_t W, const float* mean, const float* stdv, void* stream) {
  VDA_CHECK_ARG(frames && out && mean && stdv, "null pointer");
  VDA_CHECK_ARG(N > 0 && h > 0 && w > 0 && H > 0 && W > 0, "empty frame geometry");
  VDA_CHECK_ARG(H <= 65535 && N <= 65535, "output height / frame count exceed the launch grid");
  NormArgs na;
  for (int c = 0; c < 3; ++c) {
    VDA_CHECK_ARG(stdv[c] != 0.f, "std must be non-zero");
    na.mean[c] = mean[c];
    na.std_[c] = stdv[c];
  }
  hipLaunchKernelGGL(preprocess_kernel, dim3((W + 255) / 256, H, N), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)frames, out, h, w, H, W, na);
  VDA_LAUNCH_CHECK();
  return 0;
}

extern "C" int vda_depth_resize(const float* depth, float* out, int32_t N, int32_t H, int32_t W, int32_t ho,
                                int32_t wo, void* stream) {
  VDA_CHECK_ARG(depth && out, "null pointer");
  VDA_CHECK_ARG(N > 0 && H > 0 && W > 0 && ho > 0 && wo > 0, "empty depth geometry");
  VDA_CHECK_ARG(ho <= 65535 && N <= 65535, "output height / frame count exceed the launch grid");
  hipLaunchKernelGGL(depth_resize_kernel, dim3((wo + 255) / 256, ho, N), dim3(256), 0, (hipStream_t)stream, depth, out,
                     H, W, ho, wo);
  VDA_LAUNCH_CHECK();
  return 0;
}
