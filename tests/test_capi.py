"""The C-ABI library: loads, exports exactly what include/vda.h declares, validates arguments.

CPU-only: the argument checks run before any HIP call, so they are exercised without a GPU.
"""
import ctypes
import os
import re
import subprocess

import pytest

import vda_amd
from vda_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "vda.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vda_[a-z0-9_]+)\s*\(", src)))


def test_header_lists_match_binding():
    assert header_functions() == sorted(_lib.EXPORTED)


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libvda.so not built")
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (vda_[a-z0-9_]+)", out))
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing


def test_product_library_has_no_tuning_state():
    """the product libvda.so exports no vda_debug_* hook and holds no writable global
    besides the per-thread error string and the memoised CU count (a device property); the route
    knobs exist only in the tuning build (include/vda_tune.h), which exports every hook it declares."""
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libvda.so not built")
    dyn = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "vda_debug_" not in dyn
    syms = subprocess.run(["nm", _lib.LIB_PATH], capture_output=True, text=True).stdout
    data = [l.split()[-1] for l in syms.splitlines() if re.match(r"\S+ [BbDd] ", l)]
    data = [d for d in data if not re.search(r"kernel|__hip|fatbin|__dso|_DYNAMIC|_GLOBAL_OFFSET|__do_|__init|__fini", d)]
    assert sorted(data) == sorted(["_ZN12_GLOBAL__N_15g_errE", "_ZZ12vda_cu_countvE3cus"]), data
    tune_h = open(os.path.join(REPO, "include", "vda_tune.h")).read()
    tune_h = re.sub(r"/\*.*?\*/", "", tune_h, flags=re.S)
    declared = sorted(set(re.findall(r"\b(vda_[a-z0-9_]+)\s*\(", tune_h)))
    assert declared == sorted(_lib.TUNE_EXPORTED)
    if os.path.exists(_lib.TUNE_LIB_PATH):
        tdyn = subprocess.run(["nm", "-D", "--defined-only", _lib.TUNE_LIB_PATH], capture_output=True, text=True).stdout
        assert set(re.findall(r"\bT (vda_debug_[a-z0-9_]+)", tdyn)) == set(declared)


def test_integration_doc_binding_matches_library():
    """INTEGRATION.md's ctypes stub is what a maintainer copies: its Epilogue mirror must have the
    library's sizeof(vda_epilogue) and the field order of _lib.Epilogue (a short struct makes
    vda_gemm read past it)."""
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    m = re.search(r"class Epilogue\(ctypes\.Structure\):.*?_fields_ = (\[.*?\])\n", doc, re.S)
    assert m, "INTEGRATION.md has no Epilogue mirror"
    fields = eval(m.group(1), {"ctypes": ctypes})  # the doc's own literal, ctypes types only
    Doc = type("DocEpilogue", (ctypes.Structure,), {"_fields_": fields})
    assert [f[0] for f in fields] == [f[0] for f in _lib.Epilogue._fields_]
    assert [f[1] for f in fields] == [f[1] for f in _lib.Epilogue._fields_]
    assert ctypes.sizeof(Doc) == _lib.lib().vda_epilogue_size()
    assert "vda_epilogue_size()" in doc  # the stub checks its mirror against the library


def test_version_and_error_plumbing():
    lib = _lib.lib()
    assert b"gfx950" in lib.vda_version()
    e = _lib.Epilogue()
    rc = lib.vda_gemm(None, 8, None, None, 8, 1, 4, 8, e, None)
    assert rc == -22
    assert b"null pointer" in lib.vda_last_error()


@pytest.mark.parametrize("args,msg", [
    ((16, 0, 16, 4, 16), b"empty GEMM"),      # M, N, K, ldx/ldy variations
    ((16, 4, 12, 4, 16), b"multiples of 8"),  # K % 8
    ((16, 6, 16, 6, 16), b"multiples of 4"),  # N % 4
])
def test_gemm_argument_validation(args, msg):
    lib = _lib.lib()
    M, N, K, ldy, ldx = args
    fake = ctypes.c_void_p(0x1000)
    rc = lib.vda_gemm(fake, ldx, fake, fake, ldy, M, N, K, _lib.Epilogue(), None)
    assert rc == -22
    assert msg in lib.vda_last_error()


def test_epilogue_combinations_rejected():
    """Epilogue options no kernel route implements are rejected up front: the LN fold
    with ReLU or a row bias, row statistics with GEGLU (its output is N/2 wide) or in fp32 mode."""
    lib = _lib.lib()
    fake = ctypes.c_void_p(0x1000)
    e = _lib.Epilogue(rdiv=1, rmod=1, ln_stats=0x2000, ln_colsum=0x3000, act=_lib.ACT_RELU)
    assert lib.vda_gemm(fake, 64, fake, fake, 256, 4096, 256, 64, e, None) == -22
    assert b"ln_stats" in lib.vda_last_error()
    e = _lib.Epilogue(rdiv=1, rmod=1, ln_stats=0x2000, ln_colsum=0x3000, rowbias=0x4000)
    assert lib.vda_gemm(fake, 64, fake, fake, 256, 4096, 256, 64, e, None) == -22
    e = _lib.Epilogue(rdiv=1, rmod=1, stats_out=0x2000, act=_lib.ACT_GEGLU)
    assert lib.vda_gemm(fake, 64, fake, fake, 256, 4096, 256, 64, e, None) == -22
    assert b"stats_out" in lib.vda_last_error()
    e = _lib.Epilogue(rdiv=1, rmod=1, stats_out=0x2000)
    assert lib.vda_gemm_f32(fake, 64, fake, fake, 256, 4096, 256, 64, e, None) == -22


def test_res2_upsample_validation():
    """An upsampled res2 (vda_epilogue.res2_h/res2_w) is a conv-epilogue option of the halo-tiled
    256-channel route only: the GEMM, the fp32 conv and other conv routes reject it before any launch,
    and vda_conv2d_res2_upsample_ok answers which shapes take it (the model's 148^2 refinenet1 conv)."""
    lib = _lib.lib()
    fake = ctypes.c_void_p(0x1000)
    assert lib.vda_conv2d_res2_upsample_ok(32, 148, 148, 256, 256, 3, 1, 1) == 1
    assert lib.vda_conv2d_res2_upsample_ok(32, 148, 264, 256, 256, 3, 1, 1) == 1   # 518x924 input
    assert lib.vda_conv2d_res2_upsample_ok(32, 37, 37, 256, 256, 3, 1, 1) == 0     # implicit-GEMM route
    assert lib.vda_conv2d_res2_upsample_ok(32, 148, 148, 256, 128, 3, 1, 1) == 0   # Cout 128
    assert lib.vda_conv2d_res2_upsample_ok(32, 148, 148, 256, 256, 3, 2, 1) == 0   # stride 2
    e = _lib.Epilogue(rdiv=1, rmod=1, res2=0x2000, ldres2=256, res2_h=74, res2_w=74)
    assert lib.vda_gemm(fake, 64, fake, fake, 256, 4096, 256, 64, e, None) == -22
    assert b"vda_conv2d only" in lib.vda_last_error()
    assert lib.vda_conv2d(fake, fake, fake, 32, 37, 37, 256, 256, 3, 1, 1, 0, 0, 0, e, None, 0, None) == -22
    assert b"upsampled res2" in lib.vda_last_error()
    e.res2_h = 200  # larger than the output grid
    assert lib.vda_conv2d(fake, fake, fake, 32, 148, 148, 256, 256, 3, 1, 1, 0, 0, 0, e, None, 0, None) == -22
    e.res2_h = 74
    assert lib.vda_conv2d_f32(fake, fake, fake, 32, 148, 148, 256, 256, 3, 1, 1, 0, e, None) == -22


def test_conv_and_attention_validation():
    lib = _lib.lib()
    fake = ctypes.c_void_p(0x1000)
    e = _lib.Epilogue()
    assert lib.vda_conv2d(fake, fake, fake, 1, 8, 8, 12, 16, 3, 1, 1, 0, 0, 0, e, None, 0, None) == -22  # Cin % 8
    assert lib.vda_spatial_attention(fake, fake, 1, 10, 2, 32, 0.1, None) == -22                # D != 64
    assert lib.vda_temporal_attention(fake, fake, 1, 33, 4, 8, 16, 0.1, 0.0, None) == -22     # T > 32
    assert b"T <= 32" in lib.vda_last_error()
    assert lib.vda_patch_im2col(fake, fake, 1, 20, 28, 592, None) == -22                      # H % 14
    assert b"multiples of the patch size" in lib.vda_last_error()


def test_model_refuses_cpu_input():
    import torch
    m = vda_amd.VideoDepthAnything.from_config("vits", device="meta")
    with pytest.raises(RuntimeError, match="GPU only"):
        m(torch.zeros(1, 2, 3, 28, 28))


def test_torch_ops_registered_meta_shapes_and_no_cpu_kernel():
    """torch.ops.vda.* exist, trace shapes under the Meta key, and have no CPU kernel (no fallback)."""
    import torch
    import vda_amd.torch_ops  # noqa: F401
    x = torch.empty(100, 64, device="meta", dtype=torch.float16)
    w = torch.empty(96, 64, device="meta", dtype=torch.float16)
    assert torch.ops.vda.gemm(x, w, None, None, 1, 1, None, None, None, 0).shape == (100, 96)
    assert torch.ops.vda.gemm(x, w, None, None, 1, 1, None, None, None, 2).shape == (100, 48)
    m = torch.empty(2, 10, 12, 64, device="meta", dtype=torch.float16)
    wc = torch.empty(32, 3, 3, 64, device="meta", dtype=torch.float16)
    assert torch.ops.vda.conv2d(m, wc, 3, 2, 1, None, False, 0, None, None).shape == (2, 5, 6, 32)
    assert torch.ops.vda.layernorm(x, x.new_empty(64, dtype=torch.float32), x.new_empty(64, dtype=torch.float32),
                                   1e-6, 9).shape == (90, 64)
    img = torch.empty(2, 3, 28, 42, device="meta")
    assert torch.ops.vda.patch_im2col(img, 640, torch.float16).shape == (2 * 7, 640)
    assert torch.ops.vda.patch_im2col(img, 588, torch.float32).dtype == torch.float32
    assert torch.ops.vda.temporal_attention(torch.empty(2 * 32 * 5, 3 * 256, device="meta", dtype=torch.float16),
                                            2, 32, 5, 8, 32, rope_theta=1e4).shape == (2 * 32 * 5, 256)
    up = torch.ops.vda.conv2d(m, wc[:, :, :, :64], 3, 1, 1, None, False, 0, None, None, [20, 24])
    assert up.shape == (2, 20, 24, 32)
    o = torch.empty(100, 96, device="meta", dtype=torch.float16)
    assert torch.ops.vda.gemm.out(x, w, act=0, out=o) is not None
    assert torch.ops.vda.gemm(torch.empty(2740, 64, device="meta", dtype=torch.float16), w,
                              drop_period=1370).shape == (2738, 96)  # the two cls rows left out
    g = x.new_empty(64, dtype=torch.float32)
    assert torch.ops.vda.groupnorm_linear(x, g, g, 4, 32, 1e-6, w, None).shape == (100, 96)
    with pytest.raises(NotImplementedError):
        torch.ops.vda.upsample_bilinear(torch.zeros(1, 2, 2, 8, dtype=torch.float16), 4, 4)


def test_workspace_queries():
    """Workspaces are the caller's (no library-global device buffers): the strip conv's split
    workspace and the stride-2 conv's im2col matrix are sized by vda_conv2d_workspace, the depth head's resize workspace by
    vda_depth_head_workspace (0 when the fused kernel serves the shape)."""
    lib = _lib.lib()
    # ViT-L layer4_rn at 19^2 (32 frames, Cin 1024 -> 256): split into fp32 slices of M x 256
    n = lib.vda_conv2d_workspace(32, 19, 19, 1024, 256, 3, 1, 1)
    assert n > 0 and n % (32 * 19 * 19 * 256 * 4) == 0
    assert lib.vda_conv2d_workspace(32, 148, 148, 256, 256, 3, 1, 1) == 0   # implicit GEMM: no workspace
    # stride 2 with >= 4096 output pixels: the explicit im2col matrix [32*19*19, 9*1024] fp16
    assert lib.vda_conv2d_workspace(32, 37, 37, 1024, 256, 3, 2, 1) == 32 * 19 * 19 * 9 * 1024 * 2
    assert lib.vda_conv2d_workspace(4, 37, 37, 1024, 256, 3, 2, 1) == 0     # small M: the implicit GEMM
    assert lib.vda_depth_head_workspace(32, 296, 296, 128, 518, 518) == 0   # fused resize: none
    assert lib.vda_depth_head_workspace(2, 20, 20, 32, 518, 518) == 0   # C % 32: fused depth conv
    assert lib.vda_depth_head_workspace(2, 20, 20, 40, 518, 518) == 2 * 518 * 518 * 40 * 2  # C % 32 != 0: materialised


def test_groupnorm_linear_routes_and_validation():
    """vda_groupnorm_linear (motion_module.py:116-119): the fused kernel serves groups 32 with N = C in
    {64, 128, 256}; every other shape runs GroupNorm + GEMM through the workspace, which then also holds
    the normalised copy of x.  Invalid arguments return -22 before any launch."""
    lib = _lib.lib()
    for C in (64, 128, 256):
        assert lib.vda_groupnorm_linear_fused(C, 32, C) == 1
    assert lib.vda_groupnorm_linear_fused(256, 32, 512) == 0
    assert lib.vda_groupnorm_linear_fused(256, 16, 256) == 0
    assert lib.vda_groupnorm_linear_fused(512, 32, 512) == 0
    stats = (lib.vda_groupnorm_workspace(32, 1369, 256, 32) * 4 + 255) // 256 * 256
    fused = lib.vda_groupnorm_linear_workspace(32, 1369, 256, 32, 256)
    assert fused == stats  # the GroupNorm statistics only
    assert lib.vda_groupnorm_linear_workspace(32, 1369, 256, 32, 512) == stats + 32 * 1369 * 256 * 2  # + GN(x)
    fake = ctypes.c_void_p(0x1000)
    ws = lib.vda_groupnorm_linear_workspace(2, 100, 256, 32, 256)
    args = [fake, fake, fake, 2, 100, 256, 32, 1e-6, fake, None, fake, 256, None, fake]
    assert lib.vda_groupnorm_linear(*args, ws - 16, None) == -22
    assert b"workspace" in lib.vda_last_error()
    bad = list(args)
    bad[5] = 250  # C not a multiple of groups / 8
    assert lib.vda_groupnorm_linear(*bad, ws, None) == -22
    bad = list(args)
    bad[10] = ctypes.c_void_p(0x1008)  # y not 16-byte aligned
    assert lib.vda_groupnorm_linear(*bad, ws, None) == -22
    bad = list(args)
    bad[13] = None  # no workspace
    assert lib.vda_groupnorm_linear(*bad, ws, None) == -22
