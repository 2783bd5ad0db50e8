/*
 * libvda — MI355X (gfx950) kernels for the Video-Depth-Anything clip forward.
 *
 * C ABI: plain pointers, sizes and a hipStream_t passed as void*.  No torch types cross this
 * boundary; the Python host (video-depth-anything_amd/) hands in device pointers it owns.
 * Every entry point returns 0 on success, a negative errno-style code for an invalid argument
 * (-22) or a positive hipError_t for a launch failure; vda_last_error() returns the message.
 * Nothing here throws, allocates device memory or synchronises the stream, so every call can be
 * captured into a hipGraph.
 *
 * Conventions
 *   half   = IEEE fp16 (_Float16), float = fp32.
 *   Activations are token-major / NHWC: a [BT, h, w, C] feature map is a [BT*h*w, C] matrix.
 *   Linear / conv weights are fp16, K (input channel) contiguous; biases are fp32.
 *
 * The reference (FriedFeid/Video-Depth-Anything @ /root/reference) has no native layer or FFI:
 * its hot path is PyTorch modules.  Each entry point below names the reference code it replaces.
 */
#ifndef VDA_H
#define VDA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Epilogue activation codes for vda_gemm / vda_conv2d. */
enum {
  VDA_ACT_NONE = 0,
  VDA_ACT_GELU = 1,  /* exact erf GELU (nn.GELU, dinov2.py:61 act_layer)                 */
  VDA_ACT_GEGLU = 2, /* h * gelu(g); weight rows interleaved in 16-row blocks [h|g]      */
  VDA_ACT_RELU = 3
};

/* Store layouts for vda_gemm. */
enum {
  VDA_STORE_ROWS = 0,         /* Y[m*ldy + n]                                            */
  VDA_STORE_PIXEL_SHUFFLE = 1 /* ConvTranspose2d(k=s): n=(i*k+j)*Cout+co scattered to NHWC */
};

/*
 * Fused epilogue of a GEMM / conv tile, applied to the fp32 accumulator `acc` of output (m, n):
 *   acc = rstd[m] * (acc - mean[m] * ln_colsum[n])         (LayerNorm fold, when ln_stats is set)
 *   v = acc + bias[n] + rowbias[((m / rdiv) % rmod) * N + n]
 *   v = act(v)
 *   v = res[m*ldres + n] + res2[m*ldres2 + n] + gamma[n] * v      (each term optional)
 * then stored as fp16.  Null pointers disable a term.  With VDA_ACT_GEGLU the GEMM N counts the
 * interleaved [h|g] weight rows and the output has N/2 columns.
 */
typedef struct vda_epilogue {
  const float* bias;     /* [N] or NULL                                                */
  const float* rowbias;  /* [rmod, N] or NULL (patch-embed pos-embed, temporal PE·Wᵀ)  */
  int32_t rdiv, rmod;
  const float* gamma;    /* [N] LayerScale or NULL                                     */
  const void* res;       /* half [M, ldres] or NULL (may alias the output)             */
  int64_t ldres;
  const void* res2;      /* half [M, ldres2] or NULL                                   */
  int64_t ldres2;
  int32_t act;           /* VDA_ACT_*                                                  */
  int32_t store;         /* VDA_STORE_*                                                */
  int32_t ps_k, ps_cout, ps_hin, ps_win; /* pixel-shuffle geometry (store == 1)       */
  /* LayerNorm folded into the GEMM (block.py:84,87 norm1 / norm2 feeding qkv / fc1): X is the raw
   * row stream x, W holds gamma (.) W_ln, bias holds W_ln beta + b, ln_colsum[n] = sum_k W[n, k] (of the
   * fp16 W actually used), and ln_stats[m] = (mean, rstd) of row m from vda_row_stats.  Then
   * rstd (x W^T - mean colsum) + bias = LN(x) W_ln^T + b exactly in real arithmetic.  Row store only, no gamma, activation none / gelu.
   * With a rowbias (the motion-module q/k/v: LN(x) + pe[t] then to_q/k/v, motion_module.py:175,256,
   * 263): bias required, no activation / res / res2 / stats_out, rdiv >= 256, N % 256 == 0,
   * M >= 4096, K % 64 == 0, 16-byte aligned x / y rows (the phased route's EK 3 epilogue; -22
   * otherwise). */
  const float* ln_stats;  /* [M, 2] or NULL                                              */
  const float* ln_colsum; /* [N]                                                     */
  /* ln_parts > 0: ln_stats instead holds [M, ln_parts, 2] partial (sum, sum of squares) of row m
   * over ln_parts column blocks (as written through stats_out by the GEMM that produced X); the
   * epilogue forms mean = sum / K, var = max(sumsq / K - mean^2, 0), rstd = 1 / sqrt(var + ln_eps).
   * ln_parts <= 4, M * max(ln_parts, 1) >= 2.  No padding is needed past [M, ln_parts, 2]: the kernels
   * never read beyond it. */
  int32_t ln_parts;
  float ln_eps;
  /* Producer side: write [M, ceil(N / 256), 2] per-row partial (sum, sum of squares) of the fp16
   * OUTPUT values (after the residual adds) over 256-column blocks, for a following LN-folded GEMM
   * (ln_parts = ceil(N / 256)): the statistics pass over the row stream is never a separate read.
   * Row store, no pixel shuffle, no GEGLU; computed by a separate partial-sum kernel when the GEMM
   * shape does not take the phased 256x256 kernel (then N % 8 == 0, ldy % 8 == 0, y 16-byte aligned).
   * Not available in the fp32 entry points. */
  float* stats_out;
  /* res2_h, res2_w > 0 (vda_conv2d only): res2 is a smaller [BT, res2_h, res2_w, N] map read through a
   * bilinear align_corners=True upsample to the output grid (the FeatureFusionBlock input upsampled by
   * the previous block, blocks.py:156-158, consumed as refinenet1's skip add, blocks.py:146-150),
   * bit-identical to vda_upsample_bilinear + the add; ldres2 is then the source row stride (= N).
   * Served where vda_conv2d_res2_upsample_ok says so (the halo-tiled 256-channel conv); 0 = same grid. */
  int32_t res2_h, res2_w;
  /* Optional tile scheduler of the persistent 256x256 GEMM: 9 int32, zero before the first launch and
   * left zero by every launch (the last block to finish clears them).  Blocks then take their tiles
   * beyond the first round by atomic ticket (per XCD) instead of a fixed stride, so blocks that start
   * late (the GPU shared with another stream's kernels) run fewer tiles.  A counter set must not be used
   * by two launches that can run at the same time (one per stream).  NULL: static schedule.  Ignored by
   * the other kernel routes. */
  int32_t* sched;
  /* drop_period > 0 (vda_gemm only): X is a token stream of frames of drop_period rows whose first row is
   * the cls token (the encoder output, dinov2.py:309-312 get_intermediate_layers drops it); output rows
   * m with m % drop_period == 0 are not stored and row m goes to Y row m - m / drop_period - 1, so Y
   * holds the M - ceil(M / drop_period) patch rows.  For the DPT projects 1x1 conv on a tap with the
   * final LayerNorm folded in (dpt.py:60-68).  Served by the phased route's register epilogue only:
   * drop_period >= 256, ln_stats + ln_colsum + bias, activation none, row store, no gamma / res / res2 /
   * rowbias / stats_out, N % 256 == 0, M >= 4096, K % 64 == 0, 16-byte aligned Y rows; -22 otherwise. */
  int32_t drop_period;
} vda_epilogue;

/* Version / diagnostics. */
const char* vda_version(void);
/* sizeof(vda_epilogue) as compiled into the library (bindings check their mirror against it). */
int64_t vda_epilogue_size(void);
const char* vda_last_error(void);

/*
 * Y[M, N] = epilogue( X[M, K] · W[N, K]ᵀ ).   fp16 in/out, fp32 accumulate, MFMA 16x16x32.
 * Replaces every nn.Linear / 1x1 nn.Conv2d / ConvTranspose2d(k=s) of the hot path:
 *   dinov2_layers/attention.py:72,79 (qkv, proj); mlp.py:36-39 (fc1+GELU, fc2); block.py:84-87
 *   (ls1/ls2 LayerScale + residual); dpt.py:60-68 (projects), dpt.py:70-82 (ConvT k4s4/k2s2);
 *   blocks.py:124-126,160 (out_conv); motion_module.py:119,127 (proj_in/out + residual);
 *   motion_module.py:263,272-273 (to_q/k/v with the PE add :256 folded as a per-frame rowbias);
 *   attention.py:328 (to_out); attention.py:374-384 (GEGLU) and :338 (ff out).
 * Requires K % 8 == 0, ldx % 8 == 0, N % 4 == 0 (N % 32 == 0 for GEGLU).
 */
int vda_gemm(const void* x, int64_t ldx, const void* w, void* y, int64_t ldy,
             int32_t M, int32_t N, int32_t K, const vda_epilogue* epi, void* stream);

/*
 * NHWC implicit-GEMM 2-D convolution, fp16 MFMA, square kernel `ks`, zero padding `pad`.
 * X [BT, H, W, Cin] half; Wt [Cout, ks, ks, Cin] half; Y [BT, Ho, Wo, Cout] half.
 * pre_relu applies ReLU to X as it is loaded (ResidualConvUnit, blocks.py:78).
 * Replaces blocks.py:20-32 (layerN_rn 3x3 no bias), blocks.py:78-91 (RCU conv1/conv2 + skip
 * add), blocks.py:146-150 (fusion skip add, via res2), dpt.py:83-89 (3x3 s2 resize), and
 * dpt.py:117 (output_conv1).  Requires Cin % 8 == 0, Cout % 4 == 0.
 * If `up_h`/`up_w` > 0, X is read through a bilinear align_corners=True upsample from
 * [BT, H, W, Cin] to [BT, up_h, up_w, Cin] (blocks.py:156-158 / dpt_temporal.py:92-94), and the
 * conv runs on the upsampled grid.
 * `ws` / `ws_bytes`: a device workspace of vda_conv2d_workspace(...) bytes lets the strip-tiled
 * 3x3 kernel split small maps' input channels over several work items (fp32 partial slices summed
 * in a fixed order: deterministic).  NULL / 0 runs the same conv unsplit.  The library keeps no
 * mutable device state of its own, so calls on different streams with their own workspaces may
 * run concurrently.
 */
int vda_conv2d(const void* x, const void* w, void* y, int32_t BT, int32_t H, int32_t W,
               int32_t Cin, int32_t Cout, int32_t ks, int32_t stride, int32_t pad,
               int32_t pre_relu, int32_t up_h, int32_t up_w, const vda_epilogue* epi,
               void* ws, int64_t ws_bytes, void* stream);
int64_t vda_conv2d_workspace(int32_t BT, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t ks,
                             int32_t stride, int32_t pad);
/* 1 when vda_conv2d of this shape takes an epilogue res2 through the fused upsample (res2_h/res2_w),
 * else 0 (the caller materialises the upsample with vda_upsample_bilinear instead). */
int vda_conv2d_res2_upsample_ok(int32_t BT, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t ks,
                                int32_t stride, int32_t pad);

/*
 * Row LayerNorm, fp32 statistics.  X rows of C halfs (row stride ldx); Y [rows, C] half.
 * With skip_period > 0, output row r reads input row r + r/(skip_period) + 1, i.e. it drops the
 * cls token of every [1+skip_period]-token frame (dinov2.py:309-312).
 * Replaces block.py:84,87 (norm1/norm2, eps 1e-6), dinov2.py:310 (final norm on the taps),
 * motion_module.py:175,183 (temporal LayerNorms, eps 1e-5).
 */
int vda_layernorm(const void* x, int64_t ldx, void* y, const float* gamma, const float* beta,
                  int32_t rows, int32_t C, float eps, int32_t skip_period, void* stream);

/*
 * Per-row LayerNorm statistics for the LN-folded GEMM (vda_epilogue.ln_stats): stats[r] = (mean,
 * 1/sqrt(var + eps)) of row r of X (rows of C halfs, row stride ldx), fp32, two-pass like
 * vda_layernorm (same values).  Replaces the statistics half of block.py:84,87 (norm1 / norm2).
 */
int vda_row_stats(const void* x, int64_t ldx, float* stats, int32_t rows, int32_t C, float eps,
                  void* stream);

/*
 * GroupNorm over NHWC frames: X [F, S, C] half -> Y [F, S, C] half, `groups` groups of C/groups
 * channels, statistics over (S x C/groups) in fp32.  `ws`: a float workspace of
 * vda_groupnorm_workspace(F, S, C, groups) entries enables the three-pass coalesced path
 * (per-chunk partial sums around a per-group shift, finalize, apply; deterministic); NULL runs the
 * one-block-per-(frame, group) kernel.  Replaces motion_module.py:116 (GroupNorm(32, eps 1e-6)).
 */
int vda_groupnorm(const void* x, void* y, const float* gamma, const float* beta, int32_t F,
                  int32_t S, int32_t C, int32_t groups, float eps, float* ws, void* stream);
int64_t vda_groupnorm_workspace(int32_t F, int32_t S, int32_t C, int32_t groups);

/*
 * GroupNorm -> Linear: Y [F*S, N] = GN(X) · Wᵀ + bias, X [F, S, C] half, W [N, C] half, gamma / beta /
 * bias fp32 (bias may be NULL), Y half.  Replaces motion_module.py:116-119 (self.norm(hidden_states),
 * the (b f) c h w -> (b f) (h w) c rearrange, self.proj_in) - the op SURVEY.md §8(b) names
 * groupnorm_linear.  For groups == 32 and N == C in {64, 128, 256} (every motion module of the
 * shipped encoders) the normalisation is applied to the GEMM operand in registers (no normalised copy
 * of X in HBM): W' = fp16(W diag(gamma)) and W beta + bias are formed per block in LDS, and the operand
 * is fp16((x - mean) rstd); other shapes run vda_groupnorm + vda_gemm through the workspace
 * (vda_groupnorm_linear_fused says which; ViT-L's C = 1024 modules take this route).  stats_out
 * (optional): [F*S, ceil(N / 256), 2] per-row (sum, sum of squares) of the stored fp16 rows over
 * 256-column blocks, as vda_epilogue.stats_out.  ws: a 16-byte aligned
 * device buffer of at least vda_groupnorm_linear_workspace(...) bytes.  x, w, y 16-byte aligned.
 */
int vda_groupnorm_linear(const void* x, const float* gamma, const float* beta, int32_t F, int32_t S,
                         int32_t C, int32_t groups, float eps, const void* w, const float* bias, void* y,
                         int32_t N, float* stats_out, void* ws, int64_t ws_bytes, void* stream);
int64_t vda_groupnorm_linear_workspace(int32_t F, int32_t S, int32_t C, int32_t groups, int32_t N);
int vda_groupnorm_linear_fused(int32_t C, int32_t groups, int32_t N);

/*
 * Spatial multi-head self-attention (flash / online softmax, fp16 MFMA, fp32 softmax).
 * qkv [B*N, 3*H*D] half laid out as [B, N, 3, H, D] (the nn.Linear qkv output);
 * out [B*N, H*D] half.  D must be 64.  Replaces dinov2_layers/attention.py:49-62/:65-81
 * (softmax(q kᵀ / sqrt(D)) v; xformers memory_efficient_attention BMHK).
 */
int vda_spatial_attention(const void* qkv, void* out, int32_t B, int32_t N, int32_t H,
                          int32_t D, float scale, void* stream);

/*
 * Temporal self-attention across T <= 32 frames at every spatial site.
 * qkv [(B*T)*S, 3*H*D] half (frame-major rows, [q|k|v] columns, heads contiguous);
 * out [(B*T)*S, H*D] half.  D % 8 == 0, D <= 128.
 * rope_theta > 0 applies the rotary embedding of pe='rope' to q and k first: channel pairs
 * (2i, 2i+1) of all C = H*D channels of frame t rotate by t * rope_theta^(-2i/C), in fp32 from the
 * fp16 q/k, rounded back to fp16 (attention.py:403-429, motion_module.py:290-293); 0 = none ('ape',
 * whose additive table the caller folds into the q/k/v GEMM as a row bias).
 * Replaces motion_module.py:247-335 (rearrange (b f) d c -> (b d) f c, 8-head softmax over f,
 * rearrange back) and attention.py:182-211/:256-293.
 */
int vda_temporal_attention(const void* qkv, void* out, int32_t B, int32_t T, int32_t S,
                           int32_t H, int32_t D, float scale, float rope_theta, void* stream);

/*
 * Bilinear resize, align_corners=True, NHWC half: X [BT, H, W, C] -> Y [BT, Ho, Wo, C].
 * Replaces blocks.py:156-158 and dpt_temporal.py:92-94 where not fused into a conv.
 */
int vda_upsample_bilinear(const void* x, void* y, int32_t BT, int32_t H, int32_t W, int32_t C,
                          int32_t Ho, int32_t Wo, void* stream);

/*
 * Patch-embed im2col: images [BT, 3, H, W] float (NCHW, as VideoDepthAnything.forward receives
 * them) -> A [BT*(1+np), Kp] half with np = (H/14)*(W/14), K order (ci, ky, kx), zero-padded to
 * Kp >= 588, and an all-zero row 0 per frame for the cls token.  Followed by vda_gemm with a
 * per-token rowbias this replaces patch_embed.py:69-82 + dinov2.py:212-219 (cls cat, pos add).
 * img must be 8-byte aligned and a 16-byte aligned (vector loads / stores); -22 otherwise.
 */
int vda_patch_im2col(const float* img, void* a, int32_t BT, int32_t H, int32_t W, int32_t Kp,
                     void* stream);

/*
 * Depth head tail (dpt_temporal.py:92-99, dpt.py:118-124, video_depth.py:63-64):
 * X [BT, Hin, Win, C] half (the output_conv1 result) is bilinearly resized (align_corners=True,
 * fp16 storage like the reference's autocast interpolate), then conv3x3(C -> 32, +b1) -> ReLU ->
 * conv1x1(32 -> 1, w2, +b2) -> ReLU.  The resize is normally fused into the conv's patch staging
 * (the resized map is never written); shapes that need it materialised use the caller's workspace
 * ws [BT, Ho, Wo, C] half of vda_depth_head_workspace(...) bytes (0 = not needed: ws may be NULL).
 * The 3x3 conv keeps fp32 weights as an exact fp16 hi/lo split: w1 is half [64, 3, 3, C] with
 * rows 0..31 = fp16(w) and rows 32..63 = fp16(w - fp16(w)); both halves accumulate in fp32.
 * depth [BT, Ho, Wo] float.  C % 8 == 0.
 */
int vda_depth_head(const void* x, const void* w1, const float* b1, const float* w2,
                   const float* b2, float* depth, void* ws, int32_t BT, int32_t Hin, int32_t Win,
                   int32_t C, int32_t Ho, int32_t Wo, void* stream);
int64_t vda_depth_head_workspace(int32_t BT, int32_t Hin, int32_t Win, int32_t C, int32_t Ho, int32_t Wo);

/*
 * Frame preprocessing on the device: uint8 RGB frames [N, h, w, 3] (HWC) -> float [N, 3, H, W]
 * = (bicubic_resize(frames / 255) - mean[c]) / std[c].  Bicubic a = -0.75, half-pixel centres,
 * clamped borders, no antialias (cv2.INTER_CUBIC; torch interpolate bicubic align_corners=False).
 * mean / std: 3 floats each in HOST memory.  Replaces util/transform.py:5-157 (Resize with
 * keep_aspect_ratio / lower_bound / multiple 14 chooses H, W on the host; NormalizeImage;
 * PrepareForNet) as video_depth.py:336-361 and :140-146, :209 apply them per frame.
 */
int vda_preprocess_frames(const void* frames, float* out, int32_t N, int32_t h, int32_t w, int32_t H,
                          int32_t W, const float* mean, const float* std, void* stream);

/*
 * Depth resize to the source frame size: depth [N, H, W] float -> out [N, ho, wo] float, bilinear
 * align_corners=True.  Replaces video_depth.py:372 (infer_video_depth) and :300 (streaming).
 */
int vda_depth_resize(const float* depth, float* out, int32_t N, int32_t H, int32_t W, int32_t ho,
                     int32_t wo, void* stream);

/*
 * fp32 mode (infer_video_depth(fp32=True) / autocast off, video_depth.py:366-368): the same ops
 * with fp32 activations AND fp32 weights, fp32 accumulation on the exact-f32 MFMA
 * (v_mfma_f32_16x16x4_f32), exact-erf GELU, expf softmax.  Same layouts and epilogue contract as
 * the fp16 entry points above (vda_epilogue.res / res2 are float here).  Parity tier (i) of
 * SURVEY.md §8(d).  Requirements: K, ldx, N multiples of 4 (GEGLU: N % 32 == 0); conv Cin, Cout
 * multiples of 4; spatial attention D == 64; temporal attention T <= 32, D <= 128.
 */
int vda_gemm_f32(const float* x, int64_t ldx, const float* w, float* y, int64_t ldy,
                 int32_t M, int32_t N, int32_t K, const vda_epilogue* epi, void* stream);
int vda_conv2d_f32(const float* x, const float* w, float* y, int32_t BT, int32_t H, int32_t W,
                   int32_t Cin, int32_t Cout, int32_t ks, int32_t stride, int32_t pad,
                   int32_t pre_relu, const vda_epilogue* epi, void* stream);
int vda_layernorm_f32(const float* x, int64_t ldx, float* y, const float* gamma, const float* beta,
                      int32_t rows, int32_t C, float eps, int32_t skip_period, void* stream);
int vda_groupnorm_f32(const float* x, float* y, const float* gamma, const float* beta, int32_t F,
                      int32_t S, int32_t C, int32_t groups, float eps, void* stream);
int vda_spatial_attention_f32(const float* qkv, float* out, int32_t B, int32_t N, int32_t H,
                              int32_t D, float scale, void* stream);
int vda_temporal_attention_f32(const float* qkv, float* out, int32_t B, int32_t T, int32_t S,
                               int32_t H, int32_t D, float scale, float rope_theta, void* stream);
int vda_upsample_bilinear_f32(const float* x, float* y, int32_t BT, int32_t H, int32_t W, int32_t C,
                              int32_t Ho, int32_t Wo, void* stream);
int vda_patch_im2col_f32(const float* img, float* a, int32_t BT, int32_t H, int32_t W, int32_t Kp,
                         void* stream);
/* Depth tail in fp32: bilinear resize into ws_up [BT, Ho, Wo, C], conv3x3(C -> 32, w1 [32, 3, 3, C],
 * +b1) -> ReLU into ws_mid [BT*Ho*Wo, 32], then 1x1 (w2 [32], +b2) -> ReLU -> depth [BT, Ho, Wo]. */
int vda_depth_head_f32(const float* x, const float* w1, const float* b1, const float* w2,
                       const float* b2, float* depth, float* ws_up, float* ws_mid, int32_t BT,
                       int32_t Hin, int32_t Win, int32_t C, int32_t Ho, int32_t Wo, void* stream);

/* The tuning entry points (vda_debug_*) exist only in the tuning build of the library
 * (make tune -> build/tune/libvda.so): include/vda_tune.h.  This library keeps no mutable global
 * state; its kernel routes are the automatic ones. */

#ifdef __cplusplus
}
#endif
#endif /* VDA_H */
