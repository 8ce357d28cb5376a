"""fp32 convolution as an autograd op over the hand-written fp32-MFMA kernels (conv_f32.hip).

The reference trains in float32 end to end (imagenet-resnet50.py:56-62: no mixed-precision
policy).  `conv2d_f32` is the drop-in for `F.conv2d` in that precision: NCHW in and out (the
storage is channels_last, i.e. NHWC, which is what the kernels read), OHWI weights as the
flat parameter layout stores them (models/resnet50.py), forward / data gradient / weight
gradient all on `v_mfma_f32_16x16x4_f32` with fp32 operands and fp32 accumulation.

  forward   y  = conv(x, w) + b                          conv_f32
  dgrad     dx = conv(dy, flip(w)^T, pad R-1-p)  (s = 1)  conv_f32
            dx = scatter_s(dy @ w)                (1x1, s > 1, p = 0: ResNet-50's strided convs)
  wgrad     dw = sum_m dy[m] (x) im2col(x)[m]             wgrad_f32
"""
from __future__ import annotations

import torch

from .native import require_native


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] (any strides) -> contiguous [N, H, W, C] (free for channels_last)."""
    return t.permute(0, 2, 3, 1).contiguous()


class _ConvF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride: int, pad: int):
        N = require_native()
        xh = _nhwc(x.float())
        co, R, S, C = w.shape
        n, H, W, _ = xh.shape
        Ho, Wo = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
        y = torch.empty(n, Ho, Wo, co, dtype=torch.float32, device=x.device)
        N.conv_f32(xh, R, S, stride, pad, w.reshape(co, -1).contiguous(), b, y)
        ctx.save_for_backward(xh, w)
        ctx.conf = (stride, pad, b is not None)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        N = require_native()
        xh, w = ctx.saved_tensors
        stride, pad, has_b = ctx.conf
        co, R, S, C = w.shape
        n, H, W, _ = xh.shape
        gyh = _nhwc(gy)
        dx = dw = db = None
        if ctx.needs_input_grad[1]:
            dw = torch.zeros(co, R * S * C, dtype=torch.float32, device=gy.device)
            N.wgrad_f32(xh, R, S, stride, pad, gyh, dw)
            dw = dw.view(co, R, S, C)
        if has_b and ctx.needs_input_grad[2]:
            db = gyh.sum(dim=(0, 1, 2))
        if ctx.needs_input_grad[0]:
            # dgrad weights [C][R'][S'][co] = w[co][R-1-r'][S-1-s'][c]
            wt = w.flip(1, 2).permute(3, 1, 2, 0).reshape(C, R * S * co).contiguous()
            if stride == 1:
                dxh = torch.empty(n, H, W, C, dtype=torch.float32, device=gy.device)
                N.conv_f32(gyh, R, S, 1, R - 1 - pad, wt, None, dxh)
            elif R == 1 and S == 1 and pad == 0:
                Ho, Wo = gyh.shape[1:3]
                small = torch.empty(n, Ho, Wo, C, dtype=torch.float32, device=gy.device)
                N.conv_f32(gyh, 1, 1, 1, 0, wt, None, small)
                dxh = torch.zeros(n, H, W, C, dtype=torch.float32, device=gy.device)
                dxh[:, ::stride, ::stride] = small
            else:
                raise NotImplementedError("conv2d_f32 dgrad: strided convs other than 1x1/pad 0 "
                                          "(ResNet-50 has none)")
            dx = dxh.permute(0, 3, 1, 2)
        return dx, dw, db, None, None


def conv2d_f32(x: torch.Tensor, w_ohwi: torch.Tensor, bias=None, stride: int = 1, padding: int = 0):
    """F.conv2d(x, w_ohwi.permute(0, 3, 1, 2), bias, stride, padding) on the fp32 HIP kernels."""
    return _ConvF32.apply(x, w_ohwi, bias, int(stride), int(padding))
