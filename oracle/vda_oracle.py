"""CPU fp32 restatement of the Video-Depth-Anything clip forward — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle for the MI355X path in ``video-depth-anything_amd/``.  It is
imported only by ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py``; the product path never imports, calls or falls back to it.

It restates, in plain PyTorch-CPU fp32 functional calls, the math of the reference hot path
``VideoDepthAnything.forward`` (FriedFeid/Video-Depth-Anything, read at /root/reference) from a
reference-format ``state_dict`` (same key names).  No reference code is
imported.  Each function cites the reference lines it follows.

Pinning: ``tests/golden/*.npz`` hold outputs of the reference itself run in the build container
(``tests/golden/make_golden.py``), on the synthetic weight recipe of
``video-depth-anything_amd/weights.py``; ``tests/test_oracle.py`` checks this restatement against
them (rel-L1 <= 1e-5).  xformers is not installed, so the reference's golden outputs follow its
math-equivalent fallback attention (dinov2_layers/attention.py:49-62, motion_module.py:316-322);
xformers' own fp16 accumulation order is parity-unpinned.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

# video_depth.py:48-51 (intermediate_layer_idx) and dinov2.py:339-378 (vit_small / vit_large)
ENCODERS = {
    "vits": dict(embed_dim=384, depth=12, heads=6, taps=[2, 5, 8, 11]),
    "vitb": dict(embed_dim=768, depth=12, heads=12, taps=[2, 5, 8, 11]),
    "vitl": dict(embed_dim=1024, depth=24, heads=16, taps=[4, 11, 17, 23]),
}
PATCH = 14


def interpolate_pos_encoding(pos_embed: Tensor, H: int, W: int) -> Tensor:
    """dinov2.py:179-210.  pos_embed [1, 1+N0, C]; returns [1, 1+ph*pw, C] (fp32)."""
    npatch = (H // PATCH) * (W // PATCH)
    N0 = pos_embed.shape[1] - 1
    if npatch == N0 and H == W:  # dinov2.py:183-184 (the variable named w there is H)
        return pos_embed
    pe = pos_embed.float()
    cls_pe, patch_pe = pe[:, 0], pe[:, 1:]
    C = pe.shape[-1]
    s0 = math.sqrt(N0)
    h0, w0 = H // PATCH + 0.1, W // PATCH + 0.1  # interpolate_offset 0.1 (dinov2.py:193-194)
    patch_pe = F.interpolate(
        patch_pe.reshape(1, int(s0), int(s0), C).permute(0, 3, 1, 2),
        scale_factor=(h0 / s0, w0 / s0), mode="bicubic", antialias=False)
    assert patch_pe.shape[-2] == int(h0) and patch_pe.shape[-1] == int(w0)
    patch_pe = patch_pe.permute(0, 2, 3, 1).reshape(1, -1, C)
    return torch.cat((cls_pe.unsqueeze(0), patch_pe), dim=1)


def encoder_taps(sd: Dict[str, Tensor], enc: str, x: Tensor, return_cls: bool = False):
    """DINOv2 get_intermediate_layers(x, taps, return_class_token=True) with norm=True.

    dinov2.py:212-231 (prepare_tokens), :271-281 (blocks), :297-321 (norm + strip cls);
    block.py:82-107 eval branch; attention.py:49-62; mlp.py:35-41; layer_scale.py:27-28.
    x [BT, 3, H, W] -> 4 x [BT, ph*pw, C] (patch tokens, final-LN applied).
    """
    cfg = ENCODERS[enc]
    C, nh = cfg["embed_dim"], cfg["heads"]
    p = "pretrained."
    BT, _, H, W = x.shape
    assert H % PATCH == 0 and W % PATCH == 0  # patch_embed.py:73-74
    t = F.conv2d(x, sd[p + "patch_embed.proj.weight"], sd[p + "patch_embed.proj.bias"], stride=PATCH)
    t = t.flatten(2).transpose(1, 2)  # patch_embed.py:77-78
    t = torch.cat((sd[p + "cls_token"].expand(BT, -1, -1), t), dim=1)
    t = t + interpolate_pos_encoding(sd[p + "pos_embed"], H, W)
    N = t.shape[1]
    outs = []
    for i in range(cfg["depth"]):
        b = f"{p}blocks.{i}."
        h = F.layer_norm(t, (C,), sd[b + "norm1.weight"], sd[b + "norm1.bias"], eps=1e-6)
        qkv = F.linear(h, sd[b + "attn.qkv.weight"], sd[b + "attn.qkv.bias"])
        qkv = qkv.reshape(BT, N, 3, nh, C // nh).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0] * (C // nh) ** -0.5, qkv[1], qkv[2]
        a = (q @ k.transpose(-2, -1)).softmax(dim=-1)
        a = (a @ v).transpose(1, 2).reshape(BT, N, C)
        a = F.linear(a, sd[b + "attn.proj.weight"], sd[b + "attn.proj.bias"])
        t = t + a * sd[b + "ls1.gamma"]
        h = F.layer_norm(t, (C,), sd[b + "norm2.weight"], sd[b + "norm2.bias"], eps=1e-6)
        h = F.gelu(F.linear(h, sd[b + "mlp.fc1.weight"], sd[b + "mlp.fc1.bias"]))
        h = F.linear(h, sd[b + "mlp.fc2.weight"], sd[b + "mlp.fc2.bias"])
        t = t + h * sd[b + "ls2.gamma"]
        if i in cfg["taps"]:
            outs.append(t)
    outs = [F.layer_norm(o, (C,), sd[p + "norm.weight"], sd[p + "norm.bias"], eps=1e-6) for o in outs]
    if return_cls:  # dinov2.py:311-312: (patch tokens, cls token) per tap
        return [o[:, 1:] for o in outs], [o[:, 0] for o in outs]
    return [o[:, 1:] for o in outs]


def positional_table(C: int, max_len: int = 32) -> Tensor:
    """motion_module.py:189-203 sinusoidal table [1, max_len, C]."""
    pos = torch.arange(max_len).unsqueeze(1)
    div = torch.exp(torch.arange(0, C, 2) * (-math.log(10000.0) / C))
    pe = torch.zeros(1, max_len, C)
    pe[0, :, 0::2] = torch.sin(pos * div)
    pe[0, :, 1::2] = torch.cos(pos * div)
    return pe


def rotary(x: Tensor, theta: float = 10000.0) -> Tensor:
    """attention.py:403-429 apply_rotary_emb for x [N, T, C]: channel pairs (2i, 2i+1) of frame t
    rotate by t * theta^(-2i/C), in fp32 (restated with real arithmetic)."""
    N_, T, C = x.shape
    freqs = 1.0 / (theta ** (torch.arange(0, C, 2)[: C // 2].float() / C))
    ang = torch.outer(torch.arange(T, dtype=torch.float32), freqs)  # [T, C/2]
    cs, sn = torch.cos(ang), torch.sin(ang)
    xr = x.float().reshape(N_, T, C // 2, 2)
    a, b = xr[..., 0], xr[..., 1]
    return torch.stack([a * cs - b * sn, a * sn + b * cs], -1).reshape(N_, T, C).to(x.dtype)


def temporal_module(sd: Dict[str, Tensor], pre: str, x: Tensor, T: int) -> Tensor:
    """TemporalModule on NCHW frames x [BT, C, h, w] -> same shape.

    motion_module.py:108-133 (GroupNorm 32 eps 1e-6, proj_in, blocks, proj_out, + residual),
    :173-186 (2 x [LN eps 1e-5 -> TemporalAttention + x], LN -> GEGLU FF + x),
    :247-335 (rearrange over frames, + PE on the input of q, k AND v, 8 heads, to_out),
    attention.py:182-211 (softmax(q kᵀ * dim_head^-0.5) v), :363-384 (GEGLU), :296-338 (FF).
    """
    p = pre + "temporal_transformer."
    BT, C, h, w = x.shape
    B = BT // T
    res = x
    y = F.group_norm(x, 32, sd[p + "norm.weight"], sd[p + "norm.bias"], eps=1e-6)
    y = y.permute(0, 2, 3, 1).reshape(BT, h * w, C)
    y = F.linear(y, sd[p + "proj_in.weight"], sd[p + "proj_in.bias"])
    tb = p + "transformer_blocks.0."
    heads = 8
    dh = C // heads
    for j in range(2):
        ab = f"{tb}attention_blocks.{j}."
        n = F.layer_norm(y, (C,), sd[f"{tb}norms.{j}.weight"], sd[f"{tb}norms.{j}.bias"], eps=1e-5)
        d = n.shape[1]
        n = n.reshape(B, T, d, C).permute(0, 2, 1, 3).reshape(B * d, T, C)  # (b f) d c -> (b d) f c
        ape = (ab + "pos_encoder.pe") in sd   # pe='ape' carries the table; 'rope' has none
        if ape:
            n = n + sd[ab + "pos_encoder.pe"][:, :T]
        q = F.linear(n, sd[ab + "to_q.weight"])
        k = F.linear(n, sd[ab + "to_k.weight"])
        v = F.linear(n, sd[ab + "to_v.weight"])
        if not ape:  # motion_module.py:290-293
            q, k = rotary(q), rotary(k)

        def split(t):
            return t.reshape(B * d, T, heads, dh).permute(0, 2, 1, 3)
        q, k, v = split(q), split(k), split(v)
        a = ((q @ k.transpose(-1, -2)) * dh ** -0.5).softmax(dim=-1) @ v
        a = a.permute(0, 2, 1, 3).reshape(B * d, T, C)
        a = F.linear(a, sd[ab + "to_out.0.weight"], sd[ab + "to_out.0.bias"])
        a = a.reshape(B, d, T, C).permute(0, 2, 1, 3).reshape(BT, d, C)  # (b d) f c -> (b f) d c
        y = a + y
    n = F.layer_norm(y, (C,), sd[tb + "ff_norm.weight"], sd[tb + "ff_norm.bias"], eps=1e-5)
    hg = F.linear(n, sd[tb + "ff.net.0.proj.weight"], sd[tb + "ff.net.0.proj.bias"])
    hh, gate = hg.chunk(2, dim=-1)
    y = F.linear(hh * F.gelu(gate), sd[tb + "ff.net.2.weight"], sd[tb + "ff.net.2.bias"]) + y
    y = F.linear(y, sd[p + "proj_out.weight"], sd[p + "proj_out.bias"])
    y = y.reshape(BT, h, w, C).permute(0, 3, 1, 2)
    return y + res


def _rcu(sd, pre, x):
    """blocks.py:68-91 ResidualConvUnit (groups=1; eval BatchNorm after each conv when bn=True)."""
    def bn(o, j):
        b = f"{pre}bn{j}."
        if b + "running_var" not in sd:
            return o
        return F.batch_norm(o, sd[b + "running_mean"], sd[b + "running_var"], sd[b + "weight"], sd[b + "bias"],
                            training=False, eps=1e-5)
    o = bn(F.conv2d(F.relu(x), sd[pre + "conv1.weight"], sd[pre + "conv1.bias"], padding=1), 1)
    o = bn(F.conv2d(F.relu(o), sd[pre + "conv2.weight"], sd[pre + "conv2.bias"], padding=1), 2)
    return o + x


def _fusion(sd, pre, xs: Sequence[Tensor], size=None):
    """blocks.py:135-162 FeatureFusionBlock (align_corners=True, expand=False)."""
    out = xs[0]
    if len(xs) == 2:
        out = out + _rcu(sd, pre + "resConfUnit1.", xs[1])
    out = _rcu(sd, pre + "resConfUnit2.", out)
    if size is None:
        out = F.interpolate(out, scale_factor=2, mode="bilinear", align_corners=True)
    else:
        out = F.interpolate(out, size=size, mode="bilinear", align_corners=True)
    return F.conv2d(out, sd[pre + "out_conv.weight"], sd[pre + "out_conv.bias"])


def reassemble(sd: Dict[str, Tensor], feats: List[Tensor], ph: int, pw: int, cls=None) -> List[Tensor]:
    """DPT reassemble (dpt_temporal.py:55-69 / get_motion_features :101-131, dpt.py:60-90).
    feats: 4 x [BT, ph*pw, C] -> layer_1..4 NCHW.  With readout projections (use_clstoken,
    dpt.py:92-98, :129-132) each token is GELU(Linear([token, cls]))."""
    hp = "head."
    out = []
    for i, t in enumerate(feats):
        if (f"{hp}readout_projects.{i}.0.weight") in sd:
            rd = cls[i].unsqueeze(1).expand_as(t)
            t = F.gelu(F.linear(torch.cat((t, rd), -1), sd[f"{hp}readout_projects.{i}.0.weight"],
                                sd[f"{hp}readout_projects.{i}.0.bias"]))
        x = t.permute(0, 2, 1).reshape(t.shape[0], t.shape[-1], ph, pw)
        x = F.conv2d(x, sd[f"{hp}projects.{i}.weight"], sd[f"{hp}projects.{i}.bias"])
        if i == 0:
            x = F.conv_transpose2d(x, sd[hp + "resize_layers.0.weight"], sd[hp + "resize_layers.0.bias"], stride=4)
        elif i == 1:
            x = F.conv_transpose2d(x, sd[hp + "resize_layers.1.weight"], sd[hp + "resize_layers.1.bias"], stride=2)
        elif i == 3:
            x = F.conv2d(x, sd[hp + "resize_layers.3.weight"], sd[hp + "resize_layers.3.bias"], stride=2, padding=1)
        out.append(x)
    return out


def head_from_layers(sd: Dict[str, Tensor], l1: Tensor, l2: Tensor, l3: Tensor, l4: Tensor, ph: int, pw: int,
                     T: int, skip_tmp_block: bool = False, sel=None) -> Tensor:
    """dpt_temporal.py:71-99 (clip) and foward_single_image :181-260 (streaming): layer_3/4 carry all
    T frames; with ``sel`` (frame indices), layer_1/2 carry only the selected frames and path_3 is
    cut to ``sel`` after motion module 3 (:232-238).  Returns depth [len(sel) or BT, 1, 14ph, 14pw]."""
    mm = "head.motion_modules."
    s = "head.scratch."
    l3 = temporal_module(sd, mm + "0.", l3, T)
    l4 = temporal_module(sd, mm + "1.", l4, T)
    r1 = F.conv2d(l1, sd[s + "layer1_rn.weight"], padding=1)
    r2 = F.conv2d(l2, sd[s + "layer2_rn.weight"], padding=1)
    r3 = F.conv2d(l3, sd[s + "layer3_rn.weight"], padding=1)
    r4 = F.conv2d(l4, sd[s + "layer4_rn.weight"], padding=1)
    p4 = _fusion(sd, s + "refinenet4.", [r4], size=r3.shape[2:])
    if not skip_tmp_block:
        p4 = temporal_module(sd, mm + "2.", p4, T)
    p3 = _fusion(sd, s + "refinenet3.", [p4, r3], size=r2.shape[2:])
    p3 = temporal_module(sd, mm + "3.", p3, T)
    if sel is not None:
        p3 = p3[list(sel)]
    p2 = _fusion(sd, s + "refinenet2.", [p3, r2], size=r1.shape[2:])
    p1 = _fusion(sd, s + "refinenet1.", [p2, r1])
    o = F.conv2d(p1, sd[s + "output_conv1.weight"], sd[s + "output_conv1.bias"], padding=1)
    o = F.interpolate(o, (ph * PATCH, pw * PATCH), mode="bilinear", align_corners=True)
    o = F.relu(F.conv2d(o.float(), sd[s + "output_conv2.0.weight"], sd[s + "output_conv2.0.bias"], padding=1))
    o = F.relu(F.conv2d(o, sd[s + "output_conv2.2.weight"], sd[s + "output_conv2.2.bias"]))
    return o


def dpt_temporal_head(sd: Dict[str, Tensor], feats: List[Tensor], ph: int, pw: int, T: int,
                      skip_tmp_block: bool = False, cls=None) -> Tensor:
    """dpt_temporal.py:53-99 (+ dpt.py:47-124, blocks.py).  feats: 4 x [BT, ph*pw, C]."""
    l1, l2, l3, l4 = reassemble(sd, feats, ph, pw, cls)
    return head_from_layers(sd, l1, l2, l3, l4, ph, pw, T, skip_tmp_block)


class StreamEngine:
    """The streaming mode's two model calls (video_depth.py:66-88 forward_single_image,
    dpt_temporal.py:101-131 get_motion_features, :133-260 foward_single_image) in fp32 on the CPU,
    with the interface ``vda_amd.stream`` drives (features NCHW fp32 here)."""

    def __init__(self, sd: Dict[str, Tensor], enc: str):
        self.sd = {k: v.float().cpu() for k, v in sd.items()}
        self.enc = enc

    @torch.no_grad()
    def motion_features(self, x: Tensor):
        x = x.float().cpu()
        ph, pw = x.shape[-2] // PATCH, x.shape[-1] // PATCH
        feats, cls = encoder_taps(self.sd, self.enc, x, return_cls=True)
        return tuple(reassemble(self.sd, feats, ph, pw, cls))

    @torch.no_grad()
    def predict(self, x: Tensor, old, pred_idx, T: int, skip_tmp_block: bool = False):
        x = x.float().cpu()
        H, W = x.shape[-2:]
        ph, pw = H // PATCH, W // PATCH
        new = self.motion_features(x)
        if pred_idx is not None:
            l1 = torch.cat([old[0][list(pred_idx)], new[0]], 0)
            l2 = torch.cat([old[1][list(pred_idx)], new[1]], 0)
            sel = list(pred_idx) + [T - 1]
        else:
            l1, l2, sel = new[0], new[1], [T - 1]
        l3 = torch.cat([old[2], new[2]], 0)
        l4 = torch.cat([old[3], new[3]], 0)
        d = head_from_layers(self.sd, l1, l2, l3, l4, ph, pw, T, skip_tmp_block, sel=sel)
        d = F.relu(F.interpolate(d, size=(H, W), mode="bilinear", align_corners=True))
        return d[:, 0], new


@torch.no_grad()
def forward(sd: Dict[str, Tensor], enc: str, x: Tensor, skip_tmp_block: bool = False) -> Tensor:
    """video_depth.py:58-65.  x [B, T, 3, H, W] fp32 -> depth [B, T, H, W] fp32 (CPU)."""
    sd = {k: v.float().cpu() for k, v in sd.items()}
    x = x.float().cpu()
    B, T, _, H, W = x.shape
    ph, pw = H // PATCH, W // PATCH
    feats, cls = encoder_taps(sd, enc, x.flatten(0, 1), return_cls=True)
    d = dpt_temporal_head(sd, feats, ph, pw, T, skip_tmp_block, cls)
    d = F.interpolate(d, size=(H, W), mode="bilinear", align_corners=True)
    return F.relu(d).squeeze(1).unflatten(0, (B, T))


class TorchIO:
    """Frame preprocessing and depth resize in torch fp32 (the checker for libvda's
    vda_preprocess_frames / vda_depth_resize).  util/transform.py:5-157 as applied in
    video_depth.py:336-361 (frame / 255, Resize with INTER_CUBIC, NormalizeImage, PrepareForNet) and
    video_depth.py:372 / :300 (bilinear align_corners=True back to the frame size).  cv2 is absent,
    so its INTER_CUBIC is restated as torch bicubic (a = -0.75, align_corners=False): cv2 itself is
    parity-unpinned."""
    MEAN = (0.485, 0.456, 0.406)
    STD = (0.229, 0.224, 0.225)

    @staticmethod
    def preprocess(frames: Tensor, size) -> Tensor:
        x = frames.permute(0, 3, 1, 2).float() / 255.0
        x = F.interpolate(x, size=tuple(size), mode="bicubic", align_corners=False)
        mean = torch.tensor(TorchIO.MEAN, device=x.device).view(1, 3, 1, 1)
        std = torch.tensor(TorchIO.STD, device=x.device).view(1, 3, 1, 1)
        return (x - mean) / std

    @staticmethod
    def resize_depth(depth: Tensor, size) -> Tensor:
        return F.interpolate(depth.float().unsqueeze(1), size=tuple(size), mode="bilinear", align_corners=True)[:, 0]


def rel_l1(a: Tensor, b: Tensor) -> float:
    """Relative L1 = sum|a-b| / sum|b| (SURVEY.md §8(d) parity metric)."""
    a, b = a.double(), b.double()
    return float((a - b).abs().sum() / b.abs().sum().clamp_min(1e-30))
