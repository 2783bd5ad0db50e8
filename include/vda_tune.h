/*
 * Tuning entry points of the TUNING build of libvda (make tune -> build/tune/libvda.so, -DVDA_TUNING).
 * The product libvda.so has none of them and no mutable global state: its routes are fixed at the
 * automatic choices below (-1 / 0).  Every knob is process-global in the tuning build; it exists for
 * A/B measurements (tools/) and for the tests that check each alternative kernel route against the
 * default one.
 */
#ifndef VDA_TUNE_H
#define VDA_TUNE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* GEMM / conv tile configuration (-1 = automatic; 0 = 128x128/4 waves, 1 = 256x128/8 waves,
 * 2 = 128x64/4 waves, 3 = 256x256/8 waves; -2 / -3 = automatic tiles with the strip-tiled 3x3 conv for
 * no / every Cout = 256 shape; 9 = depth tail on a materialised resize instead of the resize fused into
 * the halo conv; 10 + cfg = implicit-GEMM depth tail). */
int vda_debug_force_tile(int32_t cfg);
/* Phased 256-row GEMM: persist_blocks > 0 launches that many persistent blocks (0 = one block per tile,
 * -1 = automatic: one per CU); stagger_ticks >= 0 forces the start delay (100 MHz ticks) of the delayed
 * half of the blocks, -1 = automatic (none), -2 = half a tile when the last round is short. */
int vda_debug_gemm_sched(int32_t persist_blocks, int32_t stagger);
/* groups > 1: every phased-GEMM block starts ((block / 8) % groups) / groups of the stagger ticks late. */
int vda_debug_gemm_desync(int32_t groups);
/* 1: the residual + row-statistics GEMMs (proj / fc2) through the register epilogue (bit-identical;
 * measured slower than the staged epilogue the product uses); 0 = staged. */
int vda_debug_gemm_epi(int32_t res_register);
/* Strip-tiled 3x3 conv: split every tile's input channels over nsplit work items (1, 2, 4, 8; must divide
 * Cin / 32); 0 = automatic. */
int vda_debug_strip_split(int32_t nsplit);
/* Halo-tiled phased 3x3 conv (Cout = 256): -1 = automatic (maps of >= 128^2 pixels), 0 = never,
 * 1 = every shape it serves. */
int vda_debug_hconv(int32_t mode);
/* Depth tail: -1 = automatic (the 2-blocks-per-CU depth conv with the resize fused), 2 = the same conv on
 * a materialised resize (bit-identical; needs the workspace), 0 = the older 8-wave halo kernels. */
int vda_debug_dconv(int32_t mode);
/* fused depth conv: the second half of its grid starts units1024 x 1024 shader cycles late (0 = off) */
int vda_debug_dconv_stagger(int32_t units1024);
/* Attention kernels: spatial 1 = the round-1 16x16x32 kernel; temporal 1 = the direct-load kernel. */
int vda_debug_attn(int32_t spatial_old, int32_t temporal_old);

#ifdef __cplusplus
}
#endif
#endif /* VDA_TUNE_H */
