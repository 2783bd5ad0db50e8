"""The tuning build of libvda (make tune -> build/tune/libvda.so, include/vda_tune.h) for the tests that
compare an alternative kernel route with the product library's automatic one.

The product libvda.so has no route knobs (no mutable global state): the tests call the product through
vda_amd.ops, and the alternative route through this second copy of the kernels, loaded side by side
(both libraries are linked -Bsymbolic) and called straight through the C ABI on torch-allocated buffers.
"""
import contextlib
import ctypes
import os

import pytest
import torch

from vda_amd import _lib

_TUNE = None


def tune_lib():
    global _TUNE
    if _TUNE is None:
        if not os.path.exists(_lib.TUNE_LIB_PATH):
            pytest.fail(f"{_lib.TUNE_LIB_PATH} not built: run `make tune` (or __graft_entry__.build())")
        _TUNE = TuneLib(_lib.TUNE_LIB_PATH)
    return _TUNE


class TuneLib:
    DEFAULTS = dict(force_tile=-1, strip_split=0, hconv=-1, dconv=-1, gemm_epi=0, attn=(0, 0), gemm_sched=(-1, -1),
                    gemm_desync=0)

    def __init__(self, path):
        self.lib = ctypes.CDLL(path)
        _lib._declare(self.lib)
        assert self.lib.vda_epilogue_size() == ctypes.sizeof(_lib.Epilogue)

    def set(self, **knobs):
        for k, v in knobs.items():
            fn = getattr(self.lib, "vda_debug_" + k)
            assert (fn(*v) if isinstance(v, tuple) else fn(v)) == 0

    @contextlib.contextmanager
    def route(self, **knobs):
        """Run the block with the given knobs (vda_debug_<name>), restoring the automatic routes after."""
        self.set(**knobs)
        try:
            yield self
        finally:
            self.set(**{k: self.DEFAULTS[k] for k in knobs})

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.lib.vda_last_error().decode()}")

    def conv2d(self, x, w, *, ks=3, stride=1, pad=1, bias=None, pre_relu=False, act=0, res=None, res2=None):
        """vda_conv2d on NHWC fp16 x [BT, H, W, Cin], w [Cout, ks, ks, Cin] (the ops.conv2d contract)."""
        BT, H, W, Cin = x.shape
        Cout = w.shape[0]
        Ho, Wo = (H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1
        y = torch.empty(BT, Ho, Wo, Cout, dtype=torch.float16, device=x.device)
        e = _lib.Epilogue(rdiv=1, rmod=1, act=act)
        if bias is not None:
            e.bias = bias.data_ptr()
        if res is not None:
            e.res, e.ldres = res.data_ptr(), Cout
        if res2 is not None:
            e.res2, e.ldres2 = res2.data_ptr(), Cout
            if tuple(res2.shape[1:3]) != (Ho, Wo):  # read through the upsample in the epilogue
                e.res2_h, e.res2_w = res2.shape[1], res2.shape[2]
        wsb = self.lib.vda_conv2d_workspace(BT, H, W, Cin, Cout, ks, stride, pad)
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=x.device)
        st = torch.cuda.current_stream().cuda_stream
        self._check(self.lib.vda_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), BT, H, W, Cin, Cout, ks, stride, pad,
                                        int(pre_relu), 0, 0, ctypes.byref(e), ws.data_ptr() if wsb > 0 else None, wsb,
                                        st), "vda_conv2d")
        return y

    def depth_head_workspace(self, BT, H, W, C, Ho, Wo):
        return self.lib.vda_depth_head_workspace(BT, H, W, C, Ho, Wo)

    def depth_head(self, x, w1_split, b1, w2, b2, Ho, Wo):
        """vda_depth_head on NHWC fp16 x [BT, H, W, C] (the ops.depth_head contract)."""
        BT, H, W, C = x.shape
        d = torch.empty(BT, Ho, Wo, dtype=torch.float32, device=x.device)
        wsb = self.depth_head_workspace(BT, H, W, C, Ho, Wo)
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=x.device)
        st = torch.cuda.current_stream().cuda_stream
        self._check(self.lib.vda_depth_head(x.data_ptr(), w1_split.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(),
                                            d.data_ptr(), ws.data_ptr() if wsb > 0 else None, BT, H, W, C, Ho, Wo, st),
                    "vda_depth_head")
        return d

    def gemm(self, x, w, y, e, M, N, K):
        st = torch.cuda.current_stream().cuda_stream
        self._check(self.lib.vda_gemm(x.data_ptr(), x.stride(0), w.data_ptr(), y.data_ptr(), y.stride(0), M, N, K,
                                      ctypes.byref(e), st), "vda_gemm")
        return y
