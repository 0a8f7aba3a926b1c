"""PyTorch autograd front-end to the gfx950 conv kernels: TF-'SAME' stride-2 5x5 conv and
conv_transpose as ``torch.autograd.Function`` s and ``nn.Module`` s, for users who want the
HIP kernels inside their own PyTorch code rather than the fused training engine.

Tensors are NHWC bf16 on the GPU, weights in the TF layouts (conv HWIO ``[5,5,ci,co]``, deconv
``[5,5,co,ci]``; reference ``distriubted_model.py:176-213``). One weight tensor serves every
GEMM: the forward and the data gradient read it in the two orientations (igemm3 ``bkn``), the
weight gradient lands directly in the TF layout (wgrad kernel), so nothing is repacked.

    y = conv2d_same(x, w, bias)               # D layers
    y = conv2d_transpose_same(x, w, (H, W))   # G layers
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..models.config import same_out, same_pads
from . import hip as H


def _plan(mode, Bn, Hin, Win, Kc, Hout, Wout, N, bkn):
    p = H.igemm_cfg_for(mode, Bn, Hin, Win, Kc, Hout, Wout, N, None, bkn)
    if p is None:
        raise ValueError("no igemm tile for this shape (N=%d, bkn=%d)" % (N, bkn))
    return p


def _bf(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).contiguous()


def _kpad(c: int) -> int:
    return -(-25 * c // 16) * 16


def _conv_narrow_k(x, wb_kn, cout, bias=None):
    """Conv with few input channels (c_dim 1 / 3): im2col rows [M][kpad] x weight [25*c][N]
    (rows >= 25*c read as zeros) on the plain-GEMM path."""
    B, Hs, Ws, c = x.shape
    kp = _kpad(c)
    col = H.im2col_s2(x, kp)
    M = col.shape[0]
    cfg, sp = _plan(2, B, 1, 1, kp, same_out(Hs), same_out(Ws), cout, True)
    y = H.gemm_plain(col, wb_kn.reshape(25 * c, cout).contiguous(), bias=bias, cfg=cfg, bkn=True, splits=sp)
    return y.reshape(B, same_out(Hs), same_out(Ws), cout), col


class _Conv2dSame(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias):
        x, wb = _bf(x), _bf(w)
        B, Hs, Ws, ci = x.shape
        co = w.shape[3]
        b = None if bias is None else bias.float().contiguous()
        if ci % 8:
            y, _ = _conv_narrow_k(x, wb, co, b)
        else:
            cfg, sp = _plan(0, B, Hs, Ws, ci, same_out(Hs), same_out(Ws), co, True)
            y = H.conv2d_same(x, wb.reshape(25, ci, co), co, bias=b, cfg=cfg, bkn=True, splits=sp)
        ctx.save_for_backward(x, wb)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        dy = _bf(dy)
        B, Hs, Ws, ci = x.shape
        co = wb.shape[3]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:  # adjoint = conv_transpose with HWIO read as [tap][N=ci][K=co]
            Ho, Wo = dy.shape[1], dy.shape[2]
            cfg, sp = _plan(1, B, Ho, Wo, co, Hs, Ws, ci, False)
            dx = H.conv2d_transpose_same(dy, wb.reshape(25, ci, co), ci, (Hs, Ws), cfg=cfg, splits=sp)
        if ctx.needs_input_grad[1]:
            if ci % 8:  # im2col rows [pixels][kpad] as the gathered operand, plain wgrad
                col = H.im2col_s2(x, _kpad(ci))
                dw = H.conv_wgrad(col, dy.reshape(-1, co), 0, mode=2)[:25 * ci].reshape(5, 5, ci, co)
            else:
                dw = H.conv_wgrad(x, dy, same_pads(Hs)[0]).reshape(5, 5, ci, co)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.float().sum((0, 1, 2))
        return dx, dw, db


class _ConvTranspose2dSame(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, out_hw):
        x, wb = _bf(x), _bf(w)
        B, Hi, Wi, ci = x.shape
        co = w.shape[2]
        Ho, Wo = out_hw
        cfg, sp = _plan(1, B, Hi, Wi, ci, Ho, Wo, co, False)
        y = H.conv2d_transpose_same(x, wb.reshape(25, co, ci), co, (Ho, Wo),
                                    bias=None if bias is None else bias.float(), cfg=cfg, splits=sp)
        ctx.save_for_backward(x, wb)
        ctx.has_bias = bias is not None
        ctx.out_hw = (Ho, Wo)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        dy = _bf(dy)
        B, Hi, Wi, ci = x.shape
        co = wb.shape[2]
        Ho, Wo = ctx.out_hw
        dx = dw = db = None
        col = None
        if ctx.needs_input_grad[0]:  # adjoint = the SAME conv, weight read as [tap][K=co][N=ci]
            if co % 8:
                dx, col = _conv_narrow_k(dy, wb, ci)
            else:
                cfg, sp = _plan(0, B, Ho, Wo, co, Hi, Wi, ci, True)
                dx = H.conv2d_same(dy, wb.reshape(25, co, ci), ci, cfg=cfg, bkn=True, splits=sp)
        if ctx.needs_input_grad[1]:
            if co % 8:
                col = H.im2col_s2(dy, _kpad(co)) if col is None else col
                dw = H.conv_wgrad(col, x.reshape(-1, ci), 0, mode=2)[:25 * co].reshape(5, 5, co, ci)
            else:
                dw = H.conv_wgrad(dy, x, same_pads(Ho)[0]).reshape(5, 5, co, ci)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.float().sum((0, 1, 2))
        return dx, dw, db, None


def conv2d_same(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """TF ``conv2d(x, w, strides=[1,2,2,1], padding='SAME') + bias`` on MFMA (NHWC, HWIO)."""
    return _Conv2dSame.apply(x, w, bias)


def conv2d_transpose_same(x: torch.Tensor, w: torch.Tensor, out_hw: Tuple[int, int],
                          bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """TF ``conv2d_transpose(x, w, output_shape, strides=[1,2,2,1]) + bias`` (w [5,5,out,in])."""
    return _ConvTranspose2dSame.apply(x, w, bias, tuple(out_hw))


class Conv2dSame(torch.nn.Module):
    """5x5 / stride-2 TF-SAME conv layer (truncated-normal init like ``distriubted_model.py:181``)."""

    def __init__(self, cin: int, cout: int, std: float = 0.02, device=None):
        super().__init__()
        w = torch.empty(5, 5, cin, cout, device=device)
        torch.nn.init.trunc_normal_(w, std=std, a=-2 * std, b=2 * std)
        self.w = torch.nn.Parameter(w)
        self.biases = torch.nn.Parameter(torch.zeros(cout, device=device))

    def forward(self, x):
        return conv2d_same(x, self.w, self.biases)


class ConvTranspose2dSame(torch.nn.Module):
    """5x5 / stride-2 TF-SAME transposed conv layer (normal init like ``distriubted_model.py:196``)."""

    def __init__(self, cin: int, cout: int, std: float = 0.02, device=None):
        super().__init__()
        self.w = torch.nn.Parameter(torch.randn(5, 5, cout, cin, device=device) * std)
        self.biases = torch.nn.Parameter(torch.zeros(cout, device=device))

    def forward(self, x, out_hw: Optional[Tuple[int, int]] = None):
        if out_hw is None:
            out_hw = (2 * x.shape[1], 2 * x.shape[2])
        return conv2d_transpose_same(x, self.w, out_hw, self.biases)
