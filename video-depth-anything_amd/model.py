"""VideoDepthAnything for MI355X: the reference module API and state_dict schema, HIP forward.

The module tree mirrors the reference's attribute names exactly
(video_depth.py:35-56, dinov2.py:44-170, dinov2_layers/*, dpt.py:47-124, dpt_temporal.py:23-51,
motion_module/*, util/blocks.py), so a reference checkpoint loads with ``strict=True``.  The
tree only *holds* parameters: ``forward`` never calls the sub-modules.  On first use on a device
the parameters are packed once into kernel-ready form (fp16 K-contiguous weights, fp32 biases,
NHWC conv weights, pixel-shuffle ConvT weights, GEGLU row interleave, the temporal
positional-encoding folded through to_q/k/v as a per-frame bias) and the whole clip forward then
runs on libvda kernels with NHWC / token-major activations.

``forward(x[B, T, 3, H, W] float, skip_tmp_block=False) -> depth[B, T, H, W] float`` matches
``VideoDepthAnything.forward`` (video_depth.py:58-65).  Inference only; fp16 compute with fp32
accumulation, statistics and depth tail (dpt_temporal.py:95-97 keeps output_conv2 in fp32).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from ._lib import ACT_GELU, ACT_GEGLU, ACT_RELU

PATCH = 14
ENCODER_CFG = {
    "vits": dict(embed_dim=384, depth=12, heads=6, taps=[2, 5, 8, 11]),
    "vitb": dict(embed_dim=768, depth=12, heads=12, taps=[2, 5, 8, 11]),
    "vitl": dict(embed_dim=1024, depth=24, heads=16, taps=[4, 11, 17, 23]),
}
# run.py:74-77 model_configs
MODEL_CONFIGS = {
    "vits": dict(encoder="vits", features=64, out_channels=[48, 96, 192, 384]),
    "vitb": dict(encoder="vitb", features=128, out_channels=[96, 192, 384, 768]),
    "vitl": dict(encoder="vitl", features=256, out_channels=[256, 512, 1024, 1024]),
}


# ---------------------------------------------------------------------------------------------
# Parameter-holding module tree (names == reference state_dict keys)
# ---------------------------------------------------------------------------------------------
class LayerScale(nn.Module):  # layer_scale.py:16-28
    def __init__(self, dim):
        super().__init__()
        self.gamma = nn.Parameter(torch.ones(dim))


class Attention(nn.Module):  # dinov2_layers/attention.py:29-47
    def __init__(self, dim, heads):
        super().__init__()
        self.num_heads = heads
        self.qkv = nn.Linear(dim, 3 * dim, bias=True)
        self.proj = nn.Linear(dim, dim, bias=True)


class Mlp(nn.Module):  # mlp.py:17-33
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)


class Block(nn.Module):  # block.py:36-80
    def __init__(self, dim, heads):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, heads)
        self.ls1 = LayerScale(dim)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, 4 * dim)
        self.ls2 = LayerScale(dim)


class PatchEmbed(nn.Module):  # patch_embed.py:26-67
    def __init__(self, dim):
        super().__init__()
        self.proj = nn.Conv2d(3, dim, kernel_size=PATCH, stride=PATCH)


class DinoVisionTransformer(nn.Module):  # dinov2.py:44-170, DINOv2() factory :398-415
    def __init__(self, encoder):
        super().__init__()
        cfg = ENCODER_CFG[encoder]
        C = cfg["embed_dim"]
        self.embed_dim = C
        self.num_heads = cfg["heads"]
        self.patch_size = PATCH
        self.patch_embed = PatchEmbed(C)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, C))
        self.pos_embed = nn.Parameter(torch.zeros(1, (518 // PATCH) ** 2 + 1, C))
        self.blocks = nn.ModuleList([Block(C, cfg["heads"]) for _ in range(cfg["depth"])])
        self.norm = nn.LayerNorm(C, eps=1e-6)
        self.mask_token = nn.Parameter(torch.zeros(1, C))


class ResidualConvUnit(nn.Module):  # blocks.py:37-66
    def __init__(self, f, bn=False):
        super().__init__()
        self.bn = bn
        self.conv1 = nn.Conv2d(f, f, 3, 1, 1, bias=True)
        self.conv2 = nn.Conv2d(f, f, 3, 1, 1, bias=True)
        if bn:  # blocks.py:60-62 (eval mode: folded into the convs when packing)
            self.bn1 = nn.BatchNorm2d(f)
            self.bn2 = nn.BatchNorm2d(f)


class FeatureFusionBlock(nn.Module):  # blocks.py:94-133
    def __init__(self, f, bn=False):
        super().__init__()
        self.out_conv = nn.Conv2d(f, f, 1, 1, 0, bias=True)
        self.resConfUnit1 = ResidualConvUnit(f, bn)
        self.resConfUnit2 = ResidualConvUnit(f, bn)


class PositionalEncoding(nn.Module):  # motion_module.py:189-207
    def __init__(self, d_model, max_len=32):
        super().__init__()
        pos = torch.arange(max_len).unsqueeze(1)
        div = torch.exp(torch.arange(0, d_model, 2) * (-math.log(10000.0) / d_model))
        pe = torch.zeros(1, max_len, d_model)
        pe[0, :, 0::2] = torch.sin(pos * div)
        pe[0, :, 1::2] = torch.cos(pos * div)
        self.register_buffer("pe", pe)


class TemporalAttention(nn.Module):  # motion_module.py:210-245 over attention.py:30-92
    def __init__(self, dim, max_len, pe="ape"):
        super().__init__()
        self.heads = 8
        self.pos_embedding_type = pe
        self.to_q = nn.Linear(dim, dim, bias=False)
        self.to_k = nn.Linear(dim, dim, bias=False)
        self.to_v = nn.Linear(dim, dim, bias=False)
        self.to_out = nn.ModuleList([nn.Linear(dim, dim), nn.Dropout(0.0)])
        # 'ape': sinusoidal table added before q/k/v (a state_dict buffer); 'rope': rotary q/k over
        # channel pairs with frequencies computed on the fly (attention.py:403-429; no buffer)
        self.pos_encoder = PositionalEncoding(dim, max_len) if pe == "ape" else None


class GEGLU(nn.Module):  # attention.py:363-384
    def __init__(self, dim, inner):
        super().__init__()
        self.proj = nn.Linear(dim, 2 * inner)


class FeedForward(nn.Module):  # attention.py:296-338
    def __init__(self, dim):
        super().__init__()
        self.net = nn.ModuleList([GEGLU(dim, 4 * dim), nn.Dropout(0.0), nn.Linear(4 * dim, dim)])


class TemporalTransformerBlock(nn.Module):  # motion_module.py:136-170
    def __init__(self, dim, max_len, pe="ape"):
        super().__init__()
        self.attention_blocks = nn.ModuleList([TemporalAttention(dim, max_len, pe) for _ in range(2)])
        self.norms = nn.ModuleList([nn.LayerNorm(dim) for _ in range(2)])
        self.ff = FeedForward(dim)
        self.ff_norm = nn.LayerNorm(dim)


class TemporalTransformer3DModel(nn.Module):  # motion_module.py:72-106
    def __init__(self, C, max_len, pe="ape"):
        super().__init__()
        self.norm = nn.GroupNorm(32, C, eps=1e-6, affine=True)
        self.proj_in = nn.Linear(C, C)
        self.transformer_blocks = nn.ModuleList([TemporalTransformerBlock(C, max_len, pe)])
        self.proj_out = nn.Linear(C, C)


class TemporalModule(nn.Module):  # motion_module.py:32-69 (num_transformer_block=1, dpt_temporal.py:35-40)
    def __init__(self, C, max_len=32, pe="ape"):
        super().__init__()
        self.temporal_transformer = TemporalTransformer3DModel(C, max_len, pe)


class DPTHeadTemporal(nn.Module):  # dpt.py:47-124 + dpt_temporal.py:23-51
    def __init__(self, in_channels, features, out_channels, num_frames=32, pe="ape", use_bn=False,
                 use_clstoken=False):
        super().__init__()
        self.use_clstoken = use_clstoken
        self.projects = nn.ModuleList([nn.Conv2d(in_channels, oc, 1) for oc in out_channels])
        if use_clstoken:  # dpt.py:92-98: Linear(2C -> C) + GELU on [patch token, cls token]
            self.readout_projects = nn.ModuleList([
                nn.Sequential(nn.Linear(2 * in_channels, in_channels), nn.GELU()) for _ in out_channels])
        self.resize_layers = nn.ModuleList([
            nn.ConvTranspose2d(out_channels[0], out_channels[0], 4, 4, 0),
            nn.ConvTranspose2d(out_channels[1], out_channels[1], 2, 2, 0),
            nn.Identity(),
            nn.Conv2d(out_channels[3], out_channels[3], 3, 2, 1),
        ])
        s = nn.Module()
        s.layer1_rn = nn.Conv2d(out_channels[0], features, 3, 1, 1, bias=False)
        s.layer2_rn = nn.Conv2d(out_channels[1], features, 3, 1, 1, bias=False)
        s.layer3_rn = nn.Conv2d(out_channels[2], features, 3, 1, 1, bias=False)
        s.layer4_rn = nn.Conv2d(out_channels[3], features, 3, 1, 1, bias=False)
        s.refinenet1 = FeatureFusionBlock(features, use_bn)
        s.refinenet2 = FeatureFusionBlock(features, use_bn)
        s.refinenet3 = FeatureFusionBlock(features, use_bn)
        s.refinenet4 = FeatureFusionBlock(features, use_bn)
        s.output_conv1 = nn.Conv2d(features, features // 2, 3, 1, 1)
        s.output_conv2 = nn.Sequential(nn.Conv2d(features // 2, 32, 3, 1, 1), nn.ReLU(True),
                                       nn.Conv2d(32, 1, 1, 1, 0), nn.ReLU(True), nn.Identity())
        self.scratch = s
        self.motion_modules = nn.ModuleList([
            TemporalModule(out_channels[2], num_frames, pe), TemporalModule(out_channels[3], num_frames, pe),
            TemporalModule(features, num_frames, pe), TemporalModule(features, num_frames, pe)])


# ---------------------------------------------------------------------------------------------
# Packed (kernel-ready) weights
# ---------------------------------------------------------------------------------------------
def _f(t):
    return t.detach().to(torch.float32).contiguous()


def _geglu_interleave(t):
    """Rows [h(0..I-1); g(0..I-1)] -> 16-row blocks [h(16p..16p+15); g(16p..16p+15)] (vda.h GEGLU)."""
    inner = t.shape[0] // 2
    hh, gg = t[:inner], t[inner:]
    blocks = []
    for p in range(0, inner, 16):
        blocks += [hh[p:p + 16], gg[p:p + 16]]
    return torch.cat(blocks, 0)


class _Packed:
    pass


class VideoDepthAnything(nn.Module):
    """Reference-compatible constructor (video_depth.py:36-45) and forward (:58-65).

    Per-instance schedule switches (A/B experiments only; set before the first forward, they are part
    of the packed-weight cache key): ``fold_layernorms`` folds the encoder's norm1 / norm2 into the
    qkv / fc1 GEMMs and the motion modules' attention-block LayerNorms into their q/k/v GEMMs (fp16
    mode), ``epilogue_stats`` takes those LayerNorms' row statistics from the
    proj / fc2 epilogues instead of a separate pass, ``fold_ff_norm`` folds the motion modules' ff_norm into
    their GEGLU GEMM (fp16 mode, with ``fold_layernorms``), ``fuse_groupnorm_linear`` runs each motion
    module's GroupNorm + proj_in as the one ``groupnorm_linear`` op (the normalised input never written),
    ``fold_tap_norm`` folds the final LayerNorm of each encoder tap into its DPT projects GEMM (the cls rows
    dropped in that GEMM's store), ``dynamic_tiles`` lets the encoder's persistent GEMMs
    take their tiles by atomic ticket (per-stream counters, ``ops.sched_counters``) instead of a fixed
    stride.  No environment variable changes the schedule."""

    fold_layernorms: bool = True
    epilogue_stats: bool = True
    dynamic_tiles: bool = False
    fold_ff_norm: bool = False  # built and tested; same-box forward A/B 693.7 -> 690.0 frames/s (r06_ab_ffold.log)
    fuse_groupnorm_linear: bool = True
    fold_tap_norm: bool = True

    def __init__(self, encoder="vitl", features=256, out_channels=(256, 512, 1024, 1024), use_bn=False,
                 use_clstoken=False, num_frames=32, pe="ape"):
        super().__init__()
        if pe not in ("ape", "rope"):
            raise NotImplementedError(pe)  # motion_module.py:243-244
        self.pe = pe
        self.use_bn, self.use_clstoken = bool(use_bn), bool(use_clstoken)
        self.intermediate_layer_idx = {k: v["taps"] for k, v in ENCODER_CFG.items()}
        self.encoder = encoder
        self.num_frames = num_frames
        self.features = features
        self.out_channels = list(out_channels)
        self.pretrained = DinoVisionTransformer(encoder)
        self.head = DPTHeadTemporal(self.pretrained.embed_dim, features, self.out_channels, num_frames, pe,
                                    self.use_bn, self.use_clstoken)
        self._packed: Dict[str, _Packed] = {}
        self._pos_cache: Dict[tuple, torch.Tensor] = {}

    @classmethod
    def from_config(cls, encoder: str, device="meta", pe: str = "ape", use_bn: bool = False,
                    use_clstoken: bool = False):
        """Build without running torch's default initialisers (weights are loaded afterwards)."""
        with torch.device(device):
            m = cls(**MODEL_CONFIGS[encoder], pe=pe, use_bn=use_bn, use_clstoken=use_clstoken)
        return m

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        self._packed.clear()
        self._pos_cache.clear()
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    # -- packing ---------------------------------------------------------------------------
    @torch.no_grad()
    def _pack(self, device, fp32: bool = False) -> _Packed:
        """Kernel-ready weights for ``device``: fp16 (the shipped mode) or, with ``fp32``, fp32 copies
        for the fp32-mode kernels (same layouts, vda.h *_f32)."""
        key = f"{device}|{'f32' if fp32 else 'f16'}|{int(bool(self.fold_layernorms))}"
        if key in self._packed:
            return self._packed[key]
        dev = torch.device(device)
        wd = torch.float32 if fp32 else torch.float16
        _h = lambda t: t.detach().to(wd).contiguous()  # noqa: E731  (weight storage dtype)
        _conv_nhwc = lambda w: _h(w.detach().permute(0, 2, 3, 1))  # noqa: E731  [Cout, kh, kw, Cin]
        P = _Packed()
        P.fp32, P.dt = fp32, wd
        enc = self.pretrained
        C = enc.embed_dim
        P.C, P.heads = C, enc.num_heads
        # 588 = 3*14*14 zero-padded to a multiple of 64 (the LDS-DMA GEMM K step); fp32 GEMM: K % 4
        P.Kp = 588 if fp32 else 640
        wpe = enc.patch_embed.proj.weight.reshape(C, -1)
        P.patch_w = _h(F.pad(wpe, (0, P.Kp - wpe.shape[1]))).to(dev)
        P.patch_b = _f(enc.patch_embed.proj.bias).to(dev)
        P.cls = _f(enc.cls_token.reshape(C)).to(dev)
        P.pos = _f(enc.pos_embed).to(dev)
        P.blocks = []
        # fp16 mode folds norm1 / norm2 into the qkv / fc1 GEMMs (block.py:84,87): W' = gamma (.) W,
        # b' = W beta + b, colsum = sum_k W' (of the fp16 W' the kernel multiplies); the GEMM epilogue
        # applies rstd * (x W'^T - mean colsum) + b' from per-row statistics (vda_row_stats), so the
        # normalised copy of the token tensor is never written or re-read.
        P.lnfold = not fp32 and bool(self.fold_layernorms)

        def _ln_fold(weight, bias, ln):
            w = weight.detach().float()
            wg = (w * ln.weight.detach().float()[None, :]).to(wd).contiguous()
            c1 = wg.float().sum(1).contiguous()
            bb = (w @ ln.bias.detach().float() + bias.detach().float()).contiguous()
            return wg.to(dev), c1.to(dev), bb.to(dev)

        for b in enc.blocks:
            q = _Packed()
            q.n1w, q.n1b = _f(b.norm1.weight).to(dev), _f(b.norm1.bias).to(dev)
            if P.lnfold:
                q.qkv_w, q.qkv_c1, q.qkv_b = _ln_fold(b.attn.qkv.weight, b.attn.qkv.bias, b.norm1)
            else:
                q.qkv_w, q.qkv_b = _h(b.attn.qkv.weight).to(dev), _f(b.attn.qkv.bias).to(dev)
            # LayerScale folded into the projections (gamma * (W h + b) = (gamma W) h + gamma b): the
            # GEMM epilogue then carries no per-channel multiply (block.py ls1 / ls2)
            g1 = b.ls1.gamma.detach().float()
            q.proj_w = _h(b.attn.proj.weight.detach().float() * g1[:, None]).to(dev)
            q.proj_b = _f(b.attn.proj.bias.detach().float() * g1).to(dev)
            q.n2w, q.n2b = _f(b.norm2.weight).to(dev), _f(b.norm2.bias).to(dev)
            if P.lnfold:
                q.fc1_w, q.fc1_c1, q.fc1_b = _ln_fold(b.mlp.fc1.weight, b.mlp.fc1.bias, b.norm2)
            else:
                q.fc1_w, q.fc1_b = _h(b.mlp.fc1.weight).to(dev), _f(b.mlp.fc1.bias).to(dev)
            g2 = b.ls2.gamma.detach().float()
            q.fc2_w = _h(b.mlp.fc2.weight.detach().float() * g2[:, None]).to(dev)
            q.fc2_b = _f(b.mlp.fc2.bias.detach().float() * g2).to(dev)
            P.blocks.append(q)
        P.nw, P.nb = _f(enc.norm.weight).to(dev), _f(enc.norm.bias).to(dev)

        hd = self.head
        if self.use_clstoken:  # readout Linear(2C -> C): [patch | cls] halves (dpt.py:92-98, :129-132)
            P.ro_wa, P.ro_wb, P.ro_b = [], [], []
            for rp in hd.readout_projects:
                w = rp[0].weight.detach().float()
                P.ro_wa.append(_h(w[:, :C]).to(dev))
                P.ro_wb.append(w[:, C:].contiguous().to(dev))  # fp32: the per-frame cls term, exact
                P.ro_b.append(_f(rp[0].bias).to(dev))
        P.proj_w = [_h(c.weight.reshape(c.weight.shape[0], -1)).to(dev) for c in hd.projects]
        P.proj_b = [_f(c.bias).to(dev) for c in hd.projects]
        # the final LayerNorm of each tap (dinov2.py:310) folded into its projects 1x1 conv (dpt.py:60-68)
        # the same way: the tap's normalised copy is never written (used when _tap_fold says so)
        if P.lnfold and not self.use_clstoken:
            P.projf = [_ln_fold(c.weight.reshape(c.weight.shape[0], -1), c.bias, enc.norm) for c in hd.projects]
        P.rs_w, P.rs_b = {}, {}
        for i, k in ((0, 4), (1, 2)):
            ct = hd.resize_layers[i]
            w = ct.weight  # [Cin, Cout, k, k] -> rows (i, j, co), K = Cin
            P.rs_w[i] = _h(w.permute(2, 3, 1, 0).reshape(k * k * w.shape[1], w.shape[0])).to(dev)
            P.rs_b[i] = _f(ct.bias.repeat(k * k)).to(dev)
        P.rs_w[3] = _conv_nhwc(hd.resize_layers[3].weight).to(dev)
        P.rs_b[3] = _f(hd.resize_layers[3].bias).to(dev)
        s = hd.scratch
        P.rn = [_conv_nhwc(getattr(s, f"layer{i}_rn").weight).to(dev) for i in range(1, 5)]
        P.ref = {}
        for i in range(1, 5):
            r = getattr(s, f"refinenet{i}")
            q = _Packed()
            q.out_w, q.out_b = _h(r.out_conv.weight.reshape(r.out_conv.weight.shape[0], -1)).to(dev), _f(r.out_conv.bias).to(dev)
            for u in (1, 2):
                rcu = getattr(r, f"resConfUnit{u}")
                for c in (1, 2):
                    conv = getattr(rcu, f"conv{c}")
                    w, b = conv.weight.detach().float(), conv.bias.detach().float()
                    if rcu.bn:  # eval BatchNorm after the conv (blocks.py:79-85), folded exactly in fp32
                        bnm = getattr(rcu, f"bn{c}")
                        sc = bnm.weight.detach().float() / torch.sqrt(bnm.running_var.detach().float() + bnm.eps)
                        w = w * sc[:, None, None, None]
                        b = (b - bnm.running_mean.detach().float()) * sc + bnm.bias.detach().float()
                    setattr(q, f"r{u}c{c}_w", _conv_nhwc(w).to(dev))
                    setattr(q, f"r{u}c{c}_b", _f(b).to(dev))
            P.ref[i] = q
        P.oc1_w, P.oc1_b = _conv_nhwc(s.output_conv1.weight).to(dev), _f(s.output_conv1.bias).to(dev)
        oc2 = s.output_conv2
        w1 = oc2[0].weight.detach().float().permute(0, 2, 3, 1)  # [32, 3, 3, C]
        if fp32:
            P.oc2_w1 = w1.contiguous().to(dev)
        else:
            w1_hi = w1.half()
            w1_lo = (w1 - w1_hi.float()).half()  # exact fp16 hi/lo split of the fp32 weights
            P.oc2_w1 = torch.cat([w1_hi, w1_lo], 0).contiguous().to(dev)  # [64, 3, 3, C] fp16
        P.oc2_b1 = _f(oc2[0].bias).to(dev)
        P.oc2_w2 = _f(oc2[2].weight.reshape(-1)).to(dev)
        P.oc2_b2 = _f(oc2[2].bias).to(dev)

        P.mm = []
        for m in hd.motion_modules:
            tt = m.temporal_transformer
            q = _Packed()
            Cm = tt.proj_in.weight.shape[0]
            q.C = Cm
            q.gnw, q.gnb = _f(tt.norm.weight).to(dev), _f(tt.norm.bias).to(dev)
            q.pin_w, q.pin_b = _h(tt.proj_in.weight).to(dev), _f(tt.proj_in.bias).to(dev)
            q.pout_w, q.pout_b = _h(tt.proj_out.weight).to(dev), _f(tt.proj_out.bias).to(dev)
            blk = tt.transformer_blocks[0]
            q.attn = []
            for ab, nrm in zip(blk.attention_blocks, blk.norms):
                a = _Packed()
                a.nw, a.nb = _f(nrm.weight).to(dev), _f(nrm.bias).to(dev)
                wqkv = torch.cat([ab.to_q.weight, ab.to_k.weight, ab.to_v.weight], 0).float()
                a.qkv_w = _h(wqkv).to(dev)
                # (n + pe[t]) Wᵀ = n Wᵀ + pe[t] Wᵀ: the PE add (motion_module.py:255-256) becomes a
                # per-frame fp32 row bias of the fused q/k/v GEMM.  'rope' rotates q/k inside the
                # temporal attention kernel instead (motion_module.py:290-293).
                a.pe_bias = (_f(ab.pos_encoder.pe[0].float() @ wqkv.t()).to(dev)  # [max_len, 3C]
                             if ab.pos_encoder is not None else None)
                # the LayerNorm folded into that GEMM (fp16, 'ape'; the forward takes it when a frame
                # spans >= 256 rows): W' = gamma (.) W, colsum of the fp16 W', b' = W beta
                a.fold = not fp32 and bool(self.fold_layernorms) and a.pe_bias is not None and (3 * Cm) % 256 == 0
                if a.fold:
                    a.qkv_wg = (wqkv * nrm.weight.detach().float()[None, :]).half().contiguous().to(dev)
                    a.qkv_cs = a.qkv_wg.float().sum(1).contiguous()
                    a.qkv_bb = (wqkv @ nrm.bias.detach().float()).contiguous().to(dev)
                a.out_w, a.out_b = _h(ab.to_out[0].weight).to(dev), _f(ab.to_out[0].bias).to(dev)
                q.attn.append(a)
            q.ffnw, q.ffnb = _f(blk.ff_norm.weight).to(dev), _f(blk.ff_norm.bias).to(dev)
            q.ff1_w = _h(_geglu_interleave(blk.ff.net[0].proj.weight)).to(dev)
            q.ff1_b = _f(_geglu_interleave(blk.ff.net[0].proj.bias)).to(dev)
            # ff_norm folded into the GEGLU GEMM (fp16): W' = gamma (.) W (rows interleaved as ff1_w), colsum
            # of the fp16 W', b' = W beta + b; the statistics come from the last to_out GEMM's epilogue
            q.fffold = not fp32 and bool(self.fold_layernorms)  # (the forward also checks fold_ff_norm)
            if q.fffold:
                w1 = blk.ff.net[0].proj.weight.detach().float()
                q.ff1_wg = _geglu_interleave(w1 * blk.ff_norm.weight.detach().float()[None, :]).half().contiguous().to(dev)
                q.ff1_cs = q.ff1_wg.float().sum(1).contiguous()
                q.ff1_bb = _geglu_interleave(w1 @ blk.ff_norm.bias.detach().float()
                                             + blk.ff.net[0].proj.bias.detach().float()).contiguous().to(dev)
            q.ff2_w, q.ff2_b = _h(blk.ff.net[2].weight).to(dev), _f(blk.ff.net[2].bias).to(dev)
            P.mm.append(q)
        self._packed[key] = P
        return P

    def _token_bias(self, P: _Packed, H: int, W: int, device) -> torch.Tensor:
        """Per-token fp32 bias [1+np, C]: cls+pos[0] for the cls row, conv bias + pos for patches.
        The bicubic resize of the pos table (dinov2.py:179-210) runs once per resolution (glue)."""
        key = (H, W, str(device))
        if key in self._pos_cache:
            return self._pos_cache[key]
        pos = P.pos  # [1, 1+N0, C]
        N0 = pos.shape[1] - 1
        ph, pw = H // PATCH, W // PATCH
        if ph * pw == N0 and H == W:
            pe = pos[0]
        else:
            s0 = math.sqrt(N0)
            C = pos.shape[-1]
            pp = pos[:, 1:].reshape(1, int(s0), int(s0), C).permute(0, 3, 1, 2)
            pp = F.interpolate(pp, scale_factor=((ph + 0.1) / s0, (pw + 0.1) / s0), mode="bicubic",
                               antialias=False)
            assert pp.shape[-2:] == (ph, pw)
            pe = torch.cat([pos[0, :1], pp.permute(0, 2, 3, 1).reshape(ph * pw, C)], 0)
        tb = pe.clone()
        tb[0] += P.cls
        tb[1:] += P.patch_b
        tb = tb.contiguous()
        self._pos_cache[key] = tb
        return tb

    @torch.no_grad()
    def prepare(self, device, size, fp32: bool = False) -> None:
        """Build, on the current stream, the state a forward at net input ``size`` = (H, W) would
        create lazily: the packed weights and the token bias of that resolution.  The video driver
        calls it before it spreads windows over several streams (a side stream must not read them
        while the first forward is still writing them)."""
        P = self._pack(torch.device(device), fp32)
        self._token_bias(P, int(size[0]), int(size[1]), torch.device(device))

    # -- forward ---------------------------------------------------------------------------
    def _temporal(self, q: _Packed, x: torch.Tensor, B: int, T: int, S: int) -> torch.Tensor:
        """TemporalModule on token-major frames x [B*T*S, C] (motion_module.py:64-133).
        The attention blocks' LayerNorms (motion_module.py:175) are folded into their q/k/v GEMMs when
        a frame spans >= 256 rows (each 256-row tile then sees <= 2 PE rows), and ff_norm (:182) into the
        GEGLU GEMM: the GEMM producing the residual stream h (proj_in, then each to_out) writes h's
        per-row partial sums."""
        C = q.C
        M = x.shape[0]
        fold = [a.fold and S >= 256 and M >= 4096 for a in q.attn]
        fffold = q.fffold and bool(self.fold_ff_norm)
        st = torch.empty(M + 1, (C + 255) // 256, 2, device=x.device) if any(fold) or fffold else None
        if self.fuse_groupnorm_linear:  # norm + proj_in as one op (motion_module.py:116-119)
            h = ops.groupnorm_linear(x, q.gnw, q.gnb, B * T, 32, 1e-6, q.pin_w, bias=q.pin_b,
                                     stats_out=st if fold[0] else None)
        else:
            xn = ops.groupnorm(x, q.gnw, q.gnb, B * T, 32, 1e-6)
            h = ops.gemm(xn, q.pin_w, bias=q.pin_b, stats_out=st if fold[0] else None)
        for i, a in enumerate(q.attn):
            if fold[i]:  # rstd (h W'^T - mean colsum) + W beta + pe[t] W^T
                qkv = ops.gemm(h, a.qkv_wg, bias=a.qkv_bb, rowbias=a.pe_bias, rdiv=S, rmod=T, ln_stats=st,
                               ln_parts=st.shape[1], ln_eps=1e-5, ln_colsum=a.qkv_cs)
                at = ops.temporal_attention(qkv, B, T, S, 8, C // 8)
            else:
                n = ops.layernorm(h, a.nw, a.nb, 1e-5)
                if a.pe_bias is not None:
                    qkv = ops.gemm(n, a.qkv_w, rowbias=a.pe_bias, rdiv=S, rmod=T)
                    at = ops.temporal_attention(qkv, B, T, S, 8, C // 8)
                else:  # pe='rope': rotary q/k (theta 1e4, pairs over all C channels) in the attention kernel
                    qkv = ops.gemm(n, a.qkv_w)
                    at = ops.temporal_attention(qkv, B, T, S, 8, C // 8, rope_theta=10000.0)
            # the residual-stream GEMM writes the row statistics of h for the next folded LayerNorm: the
            # next attention block's (when folded), after the last block the feed-forward's ff_norm
            nxt = fold[i + 1] if i + 1 < len(q.attn) else fffold
            h = ops.gemm(at, a.out_w, bias=a.out_b, res=h, out=h, stats_out=st if nxt else None)
        if fffold:  # rstd (h W'^T - mean colsum) + W beta + b, then the GEGLU gate (attention.py:363-384)
            g = ops.gemm(h, q.ff1_wg, bias=q.ff1_bb, act=ACT_GEGLU, ln_stats=st, ln_parts=st.shape[1], ln_eps=1e-5,
                         ln_colsum=q.ff1_cs)
        else:
            n = ops.layernorm(h, q.ffnw, q.ffnb, 1e-5)
            g = ops.gemm(n, q.ff1_w, bias=q.ff1_b, act=ACT_GEGLU)
        h = ops.gemm(g, q.ff2_w, bias=q.ff2_b, res=h, out=h)
        return ops.gemm(h, q.pout_w, bias=q.pout_b, res=x)

    def _fusion(self, q: _Packed, x0, x1, size):
        """FeatureFusionBlock (blocks.py:135-162) on NHWC maps; the 1x1 out_conv commutes with the
        bilinear resize (both linear, resize weights sum to 1), so it runs at the low resolution."""
        if x1 is not None:
            t = ops.conv2d(x1, q.r1c1_w, bias=q.r1c1_b, pre_relu=True, act=ACT_RELU)
            out = ops.conv2d(t, q.r1c2_w, bias=q.r1c2_b, res=x1, res2=x0)
        else:
            out = x0
        t = ops.conv2d(out, q.r2c1_w, bias=q.r2c1_b, pre_relu=True, act=ACT_RELU)
        out = ops.conv2d(t, q.r2c2_w, bias=q.r2c2_b, res=out)
        BT, h, w, Cf = out.shape
        y = ops.gemm(out.view(-1, Cf), q.out_w, bias=q.out_b).view(BT, h, w, Cf)
        return y, size

    def _check_input(self, x: torch.Tensor, T: int):
        if not x.is_cuda:
            raise RuntimeError("VideoDepthAnything (MI355X) runs on the GPU only; move the model input to cuda")
        Cc, H, W = x.shape[-3:]
        if Cc != 3:
            raise ValueError(f"expected 3 input channels, got {Cc}")
        if H % PATCH or W % PATCH:  # patch_embed.py:73-74
            raise AssertionError(f"Input image size ({H}x{W}) is not a multiple of the patch size {PATCH}")
        if T > self.num_frames:  # PE table length (motion_module.py:198-206)
            raise ValueError(f"clip length {T} exceeds the temporal PE table ({self.num_frames})")

    def _encode(self, P: _Packed, img: torch.Tensor):
        """DINOv2 get_intermediate_layers (dinov2.py:212-231, :271-321; block.py:104-106):
        img [BT, 3, H, W] -> (4 tap maps [BT*np, C] (final LN applied, cls row dropped),
        4 normed cls rows [BT, C] when use_clstoken else None)."""
        BT, _, H, W = img.shape
        npt = (H // PATCH) * (W // PATCH)
        ntok = npt + 1
        a = ops.patch_im2col(img.float().contiguous(), P.Kp, dtype=P.dt)
        tok = ops.gemm(a, P.patch_w, rowbias=self._token_bias(P, H, W, img.device), rdiv=1, rmod=ntok)
        del a
        taps = self.intermediate_layer_idx[self.encoder]
        feats: List[torch.Tensor] = []
        cls: Optional[List[torch.Tensor]] = [] if self.use_clstoken else None
        # LN statistics: block 0's norm1 from a row-statistics pass over the patch tokens; every later
        # norm1 / norm2 from the per-row partial sums the proj / fc2 GEMM epilogues write while they
        # update the residual stream (stats_out), so no LayerNorm reads the 90-MB token matrix again
        C = P.C
        nparts = (C + 255) // 256
        epistats = P.lnfold and nparts <= 4 and bool(self.epilogue_stats)
        if epistats:
            # [M, P, 2] exactly: the LN-folded GEMMs never read past it (vda.h ln_parts)
            st_a = torch.empty(tok.shape[0], nparts, 2, device=tok.device, dtype=torch.float32)
            st_b = torch.empty_like(st_a)
        stats, parts = None, 0
        sch = ops.sched_counters(tok.device) if self.dynamic_tiles and P.dt == torch.float16 else None
        # taps straight into their LN-folded projects GEMM, cls rows dropped in its store (vda.h drop_period)
        tapfold = epistats and self._tap_fold(P, BT, ntok)
        for i, q in enumerate(P.blocks):
            if P.lnfold:  # norm1 folded into the qkv GEMM (statistics only)
                if stats is None:
                    stats, parts = ops.row_stats(tok, 1e-6), 0
                qkv = ops.gemm(tok, q.qkv_w, bias=q.qkv_b, ln_stats=stats, ln_parts=parts, ln_eps=1e-6,
                               ln_colsum=q.qkv_c1, sched=sch)
            else:
                qkv = ops.gemm(ops.layernorm(tok, q.n1w, q.n1b, 1e-6), q.qkv_w, bias=q.qkv_b)
            at = ops.spatial_attention(qkv, BT, ntok, P.heads, 64)
            del qkv
            ops.gemm(at, q.proj_w, bias=q.proj_b, res=tok, out=tok, stats_out=st_a if epistats else None, sched=sch)
            if P.lnfold:  # norm2 folded into the fc1 GEMM
                if epistats:
                    stats, parts = st_a, nparts
                else:
                    stats, parts = ops.row_stats(tok, 1e-6), 0
                f = ops.gemm(tok, q.fc1_w, bias=q.fc1_b, act=ACT_GELU, ln_stats=stats, ln_parts=parts, ln_eps=1e-6,
                             ln_colsum=q.fc1_c1, sched=sch, tag="enc_fc1")
            else:
                f = ops.gemm(ops.layernorm(tok, q.n2w, q.n2b, 1e-6), q.fc1_w, bias=q.fc1_b, act=ACT_GELU,
                             tag="enc_fc1")
            last = i + 1 == len(P.blocks)
            ops.gemm(f, q.fc2_w, bias=q.fc2_b, res=tok, out=tok,
                     stats_out=st_b if epistats and (not last or (tapfold and i in taps)) else None, sched=sch)
            stats, parts = (st_b, nparts) if epistats else (None, 0)
            del f
            if i in taps and tapfold:  # projects(norm(tap)) with the cls rows left out (dinov2.py:309-312)
                w_, c1_, b_ = P.projf[len(feats)]
                feats.append(ops.gemm(tok, w_, bias=b_, ln_stats=st_b, ln_parts=nparts, ln_eps=1e-6, ln_colsum=c1_,
                                      drop_period=ntok))
            elif i in taps:  # final norm on the tap, cls row dropped (dinov2.py:309-312)
                feats.append(ops.layernorm(tok, P.nw, P.nb, 1e-6, skip_period=npt))
                if cls is not None:  # the same norm on each frame's cls row (row stride ntok*C)
                    cls.append(ops.layernorm(tok.view(BT, ntok, -1)[:, 0], P.nw, P.nb, 1e-6))
        return feats, cls, tapfold

    def _tap_fold(self, P: _Packed, BT: int, ntok: int) -> bool:
        """Whether the taps go straight into their LN-folded projects GEMMs: the shapes the phased GEMM's
        row-drop epilogue serves (vda.h drop_period), fp16, no readout."""
        if not (P.lnfold and bool(self.fold_tap_norm) and getattr(P, "projf", None) is not None):
            return False
        M = BT * ntok
        return (ntok >= 256 and M >= 4096 and P.C % 64 == 0 and M * P.C * 2 < 2 ** 31 and
                all(w.shape[0] % 256 == 0 and w.numel() * 2 < 2 ** 31 for w, _, _ in P.projf))

    def _reassemble(self, P: _Packed, enc, BT: int, ph: int, pw: int) -> List[torch.Tensor]:
        """DPT reassemble (dpt_temporal.py:55-69 == get_motion_features :101-131, dpt.py:60-90):
        enc = _encode's (taps, cls) -> layer_1..4 NHWC [BT, h, w, C]."""
        feats, cls, projected = enc
        oc = self.out_channels
        lay = []
        for i, ft in enumerate(feats):
            if cls is not None:
                # readout (dpt.py:129-132): GELU(W [x | cls] + b) = GELU(W_a x + (W_b cls + b)): the cls
                # term is one fp32 row per frame, a row bias of the patch GEMM
                rb = ops.gemm(cls[i].float(), P.ro_wb[i], bias=P.ro_b[i])
                ft = ops.gemm(ft, P.ro_wa[i], rowbias=rb, rdiv=ph * pw, rmod=BT, act=ACT_GELU)
            p = ft if projected else ops.gemm(ft, P.proj_w[i], bias=P.proj_b[i])
            if i == 0:
                l = ops.conv_transpose_ks(p, P.rs_w[0], P.rs_b[0], BT, ph, pw, 4)
            elif i == 1:
                l = ops.conv_transpose_ks(p, P.rs_w[1], P.rs_b[1], BT, ph, pw, 2)
            elif i == 2:
                l = p.view(BT, ph, pw, oc[2])
            else:
                l = ops.conv2d(p.view(BT, ph, pw, oc[3]), P.rs_w[3], ks=3, stride=2, pad=1, bias=P.rs_b[3])
            lay.append(l)
        return lay

    def _head(self, P: _Packed, l1, l2, l3, l4, B: int, T: int, ph: int, pw: int, skip_tmp_block: bool,
              sel: Optional[List[int]] = None) -> torch.Tensor:
        """Temporal DPT head from the reassembled maps (dpt_temporal.py:71-99).  layer_3/4 carry all
        B*T frames.  With ``sel`` (streaming, dpt_temporal.py:181-260) layer_1/2 carry only the
        selected frames and path_3 is cut to them after motion module 3.  -> depth [n, 14ph, 14pw] fp32."""
        oc = self.out_channels
        BT = B * T
        h3, w3 = l3.shape[1:3]
        h4, w4 = l4.shape[1:3]
        # temporal modules on layer_3 / layer_4 (dpt_temporal.py:75-76)
        l3 = self._temporal(P.mm[0], l3.reshape(-1, oc[2]), B, T, h3 * w3).view(BT, h3, w3, oc[2])
        l4 = self._temporal(P.mm[1], l4.reshape(-1, oc[3]), B, T, h4 * w4).view(BT, h4, w4, oc[3])
        r1 = ops.conv2d(l1, P.rn[0])
        r2 = ops.conv2d(l2, P.rn[1])
        r3 = ops.conv2d(l3, P.rn[2])
        r4 = ops.conv2d(l4, P.rn[3])
        del l1, l2, l3, l4
        Fh = self.features
        y, _ = self._fusion(P.ref[4], r4, None, None)
        p4 = ops.upsample_bilinear(y, r3.shape[1], r3.shape[2])
        if not skip_tmp_block:
            p4 = self._temporal(P.mm[2], p4.view(-1, Fh), B, T, h3 * w3).view(p4.shape)
        y, _ = self._fusion(P.ref[3], p4, r3, None)
        p3 = ops.upsample_bilinear(y, r2.shape[1], r2.shape[2])
        p3 = self._temporal(P.mm[3], p3.view(-1, Fh), B, T, p3.shape[1] * p3.shape[2]).view(p3.shape)
        if sel is not None:
            p3 = p3.index_select(0, torch.tensor(sel, dtype=torch.long, device=p3.device))
        y, _ = self._fusion(P.ref[2], p3, r2, None)
        # refinenet2's upsample to r1's grid (blocks.py:156-158) is only refinenet1's skip input (res2 of
        # its RCU conv2, blocks.py:146-150): the conv reads it through the upsample in its epilogue
        # (bit-identical; materialised by the op where the conv route has no such epilogue)
        y, _ = self._fusion(P.ref[1], y, r1, None)  # refinenet1: scale_factor 2
        H1, W1 = 2 * y.shape[1], 2 * y.shape[2]
        # refinenet1's x2 bilinear upsample (blocks.py:151-158) fused into output_conv1's patch staging
        # (fp16: the halo conv builds each patch by interpolation; fp32 mode materialises the resize)
        if P.fp32:
            o1 = ops.conv2d(ops.upsample_bilinear(y, H1, W1), P.oc1_w, bias=P.oc1_b)
        else:
            o1 = ops.conv2d(y, P.oc1_w, bias=P.oc1_b, up=(H1, W1))
        # output_conv2 with fp32 weights on the bilinear resize to (14ph, 14pw) (dpt_temporal.py:92-97);
        # the final resize to (H, W) is the identity because H = 14ph, W = 14pw (video_depth.py:63)
        if P.fp32:
            return ops.depth_head_f32(o1, P.oc2_w1, P.oc2_b1, P.oc2_w2, P.oc2_b2, ph * PATCH, pw * PATCH)
        return ops.depth_head(o1, P.oc2_w1, P.oc2_b1, P.oc2_w2, P.oc2_b2, ph * PATCH, pw * PATCH)

    @torch.no_grad()
    def forward(self, x: torch.Tensor, skip_tmp_block: bool = False, *, fp32: bool = False) -> torch.Tensor:
        """video_depth.py:58-65.  ``fp32=True`` runs every op in fp32 (the reference's forward with
        autocast off, video_depth.py:366-368); the default is fp16 compute, fp32 accumulation."""
        B, T, Cc, H, W = x.shape
        self._check_input(x, T)
        P = self._pack(x.device, fp32)
        BT = B * T
        ph, pw = H // PATCH, W // PATCH
        feats = self._encode(P, x.reshape(BT, 3, H, W))
        lay = self._reassemble(P, feats, BT, ph, pw)
        del feats
        depth = self._head(P, *lay, B, T, ph, pw, skip_tmp_block)
        return depth.view(B, T, H, W)

    # -- streaming mode (video_depth.py:66-327) ----------------------------------------------
    @torch.no_grad()
    def get_motion_features(self, x: torch.Tensor, *, fp32: bool = False):
        """Encoder + DPT reassemble of single frames (dpt_temporal.py:101-131 after
        get_intermediate_layers): x [N, 3, H, W] (or [1, N, 3, H, W]) -> (layer_1..4) NHWC fp16.
        The reference returns NCHW maps in the autocast dtype; these are the same values laid out
        for libvda."""
        if x.dim() == 5:
            x = x.flatten(0, 1)
        N, _, H, W = x.shape
        self._check_input(x, 1)
        P = self._pack(x.device, fp32)
        return tuple(self._reassemble(P, self._encode(P, x), N, H // PATCH, W // PATCH))

    @torch.no_grad()
    def forward_single_image(self, x: torch.Tensor, motion_features, pred_depth_idx=None, inference_length: int = 32,
                             skip_tmp_block: bool = False, *, fp32: bool = False):
        """video_depth.py:66-88 + dpt_temporal.py:133-260.  x [1, 1, 3, H, W]; motion_features: the
        four maps of the ``inference_length - 1`` context frames (NHWC fp16, as from
        ``get_motion_features``).  Returns (depth [1, P+1, H, W] fp32, the new frame's four maps),
        P = len(pred_depth_idx) or 0."""
        B, T1, Cc, H, W = x.shape
        T = int(inference_length)
        self._check_input(x, T)
        if B * T1 != 1:
            raise ValueError("forward_single_image takes one frame [1, 1, 3, H, W]")
        P = self._pack(x.device, fp32)
        ph, pw = H // PATCH, W // PATCH
        new = self._reassemble(P, self._encode(P, x.reshape(1, 3, H, W)), 1, ph, pw)
        o1, o2, o3, o4 = motion_features
        if o3.shape[0] + 1 != T or o4.shape[0] + 1 != T:
            raise ValueError(f"context must hold inference_length - 1 = {T - 1} frames, got {o3.shape[0]}")
        if pred_depth_idx is not None:
            pidx = [int(i) for i in pred_depth_idx]
            if pidx and not all(-o1.shape[0] <= i < o1.shape[0] for i in pidx):
                bad = next(i for i in pidx if not -o1.shape[0] <= i < o1.shape[0])
                raise IndexError(f"index {bad} is out of bounds for dimension 0 with size {o1.shape[0]}")
            it = torch.tensor(pidx, dtype=torch.long, device=x.device)
            l1 = torch.cat([o1.index_select(0, it), new[0]], 0)
            l2 = torch.cat([o2.index_select(0, it), new[1]], 0)
            sel = [i if i >= 0 else i + T for i in pidx] + [T - 1]  # path_3[idx] has T rows (:233)
        else:
            l1, l2, sel = new[0], new[1], [T - 1]
        l3 = torch.cat([o3, new[2]], 0)
        l4 = torch.cat([o4, new[3]], 0)
        depth = self._head(P, l1, l2, l3, l4, 1, T, ph, pw, skip_tmp_block, sel=sel)
        return depth.view(1, len(sel), H, W), tuple(new)

    def infere_single_image(self, frames, target_fps, input_size=518, device="cuda", fp32=False, warmup=True,
                            inference_length=32, keyframe_list=(0, 12), align_each_new_frame=True,
                            skip_tmp_block=False):
        """video_depth.py:91-327 on libvda (see vda_amd.stream); ``fp32`` selects the fp32 kernels."""
        from .stream import infere_single_image
        return infere_single_image(_StreamEngine(self, fp32), frames, target_fps, input_size=input_size, device=device,
                                   warmup=warmup, inference_length=inference_length, keyframe_list=keyframe_list,
                                   align_each_new_frame=align_each_new_frame, skip_tmp_block=skip_tmp_block)


class _StreamEngine:
    """libvda engine for vda_amd.stream: single-frame encode + head over a stored context."""

    def __init__(self, m: VideoDepthAnything, fp32: bool = False):
        self.m = m
        self.fp32 = fp32

    def motion_features(self, x):
        return self.m.get_motion_features(x, fp32=self.fp32)

    def predict(self, x, old, pred_idx, T, skip_tmp_block=False):
        d, new = self.m.forward_single_image(x.unsqueeze(0), old, pred_idx, T, skip_tmp_block, fp32=self.fp32)
        return d[0], new


def _infer_video_depth(self, frames, target_fps, input_size=518, device="cuda", fp32=False, skip_tmp_block=False,
                       windows_per_batch=1, rank=0, world=1, group=None, streams=2):
    """video_depth.py:329-417 on the MI355X forward (see vda_amd.video); ``fp32=True`` runs the
    fp32 kernels (the reference's autocast-off path), the default fp16 compute; ``streams``: window
    batches in flight on one GPU (world == 1)."""
    from .video import infer_video_depth
    return infer_video_depth(lambda x: self.forward(x, skip_tmp_block, fp32=fp32), frames, target_fps, input_size=input_size,
                             device=device, windows_per_batch=windows_per_batch, rank=rank, world=world,
                             group=group, streams=streams, prepare=lambda hw: self.prepare(device, hw, fp32))


VideoDepthAnything.infer_video_depth = _infer_video_depth


def build_model(encoder: str = "vitl", state_dict: Optional[dict] = None, device="cuda",
                pe: str = "ape", use_bn: bool = False, use_clstoken: bool = False) -> VideoDepthAnything:
    """Construct, load weights (reference checkpoint dict or the synthetic recipe), move to device."""
    from .weights import synthetic_state_dict
    m = VideoDepthAnything.from_config(encoder, device="meta", pe=pe, use_bn=use_bn, use_clstoken=use_clstoken)
    if state_dict is None:
        state_dict = synthetic_state_dict((k, tuple(v.shape)) for k, v in m.state_dict().items())
    m.load_state_dict(state_dict, strict=True, assign=True)
    m = m.to(device).eval()
    return m
