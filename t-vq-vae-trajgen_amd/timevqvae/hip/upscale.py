"""Upscale's first conv on the nearest-upsampled LF tokens, on the token grid (tvq_upscale.hip).

bidirectional_transformer.py:12-30: Upscale.forward(x (b n d), m) = conv(interpolate(x^T, m,
nearest)) with conv = Conv1d(d, H, 3, padding 1) -> GELU -> BatchNorm1d -> Conv1d.  For an
integer ratio f = m / n >= 2 the first Conv1d reads each token f times, so it is computed on
the n tokens: Z = x [W_0; W_1; W_2]^T (one GEMM, n rows instead of m), then each output
position adds the tap results of its own token and, at the token's two ends, the
neighbour's (tvq_ups_combine); its backward is the transpose (window sums of dY, two GEMMs
over n rows).  f x fewer FLOPs than upsample -> conv; equal to it up to fp32 reassociation.
"""
import contextlib

import torch

from . import streams
from ._native import call, grad_sink, ptr, stream_ptr, value
from .linear import gemm

MAX_N, MAX_M = 64, 240  # tvq_upscale.hip ups_dims_ok (LDS of the combine / sums blocks)


def supported(x, m, weight):
    """x (b, n, d) fp32 on the device, m = f n with f >= 2, weight (H, d, 3)."""
    if not x.is_cuda or x.dim() != 3 or weight.dim() != 3 or weight.shape[2] != 3:
        return False
    n = x.shape[1]
    return (n <= MAX_N and m <= MAX_M and m % n == 0 and m // n >= 2 and
            weight.shape[1] == x.shape[2] and x.dtype == torch.float32)


def _pack(w):
    H, D, _ = w.shape
    wcat = torch.empty((3 * H, D), device=w.device, dtype=torch.float32)
    call("tvq_ups_pack", ptr(w.contiguous()), H, D, ptr(wcat), stream_ptr())
    return wcat


def _z(x2, wcat):
    M, D = x2.shape
    N = wcat.shape[0]
    return gemm(x2, D, 1, wcat, 1, D, M, N, D)  # x Wcat^T (gemm_skinny)


class _UpsConvGelu(torch.autograd.Function):
    """GELU(Conv1d_k3(upsample_nearest(x^T, m)) + b) -> (b, H, m)."""

    @staticmethod
    def forward(ctx, x, w, b, m):
        B, n, D = x.shape
        H = w.shape[0]
        f = m // n
        x2 = x.reshape(B * n, D).contiguous()
        wcat = _pack(w)
        z = _z(x2, wcat)
        out = torch.empty((B, H, m), device=x.device, dtype=torch.float32)
        pre = torch.empty_like(out)
        call("tvq_ups_combine", ptr(z), B, n, f, H, ptr(b), 0, None, None, None, None, 0.0,
             ptr(out), ptr(pre), stream_ptr())
        ctx.save_for_backward(x2, wcat, pre)
        ctx.dims = (B, n, D, H, f)
        ctx.params = (w, b)
        return out

    @staticmethod
    def backward(ctx, gy):
        x2, wcat, pre = ctx.saved_tensors
        B, n, D, H, f = ctx.dims
        dev = x2.device
        g = gy.contiguous()
        need_b = ctx.params[1] is not None and ctx.needs_input_grad[2]
        s = torch.empty((B * n, 3 * H), device=dev, dtype=torch.float32)
        part = torch.empty((B, H), device=dev, dtype=torch.float32) if need_b else None
        call("tvq_ups_sums", ptr(g), ptr(pre), B, n, f, H, ptr(s), ptr(part), stream_ptr())
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = gemm(s, 3 * H, 1, wcat, D, 1, B * n, D, 3 * H).view(B, n, D)  # S Wcat
        w_p, b_p = ctx.params
        need_w = ctx.needs_input_grad[1]
        sw, sb = grad_sink(w_p), grad_sink(b_p) if b_p is not None else None
        direct = (not need_w or sw is not None) and (not need_b or sb is not None)
        if need_w or need_b:
            # into the flat gradient sinks: off the critical path (aux stream)
            with streams.offload(s, x2, part) if direct else contextlib.nullcontext():
                if need_w:
                    dwcat = gemm(s, 1, 3 * H, x2, D, 1, 3 * H, D, B * n)  # S^T x (gemm_kt)
                    dwt = sw if direct else torch.empty((H, D, 3), device=dev)
                    call("tvq_ups_wscatter", ptr(dwcat), H, D, ptr(dwt), int(direct),
                         stream_ptr())
                    if not direct:
                        dw = dwt
                if need_b:
                    dbt = sb if direct else torch.empty(H, device=dev)
                    ws = torch.empty(max(1, value("tvq_reduce_rows_workspace", B, H)), device=dev)
                    call("tvq_reduce_rows", ptr(part), B, H, H, ptr(dbt), int(direct), ptr(ws),
                         stream_ptr())
                    if not direct:
                        db = dbt
        return dx, dw, db, None


def upsample_conv_gelu(x, m, weight, bias):
    """GELU(Conv1d(interpolate(x^T, m, nearest), weight, bias, padding=1)) for x (b, n, d)
    -> (b, H, m), with autograd."""
    return _UpsConvGelu.apply(x, weight, bias, int(m))


@torch.no_grad()
def upsample_conv_gelu_bn_eval(x, m, weight, bias, bn):
    """BatchNorm1d_eval(GELU(Conv1d(interpolate(x^T, m, nearest)))) -> (b, H, m), sampling only
    (the epilogue arithmetic of tvq_conv2d_fwd_bn_eval's pre_gelu form)."""
    B, n, D = x.shape
    H = weight.shape[0]
    z = _z(x.reshape(B * n, D).contiguous(), _pack(weight))
    out = torch.empty((B, H, m), device=x.device, dtype=torch.float32)
    call("tvq_ups_combine", ptr(z), B, n, m // n, H, ptr(bias), 2, ptr(bn.weight), ptr(bn.bias),
         ptr(bn.running_mean), ptr(bn.running_var), float(bn.eps), ptr(out), None, stream_ptr())
    return out
