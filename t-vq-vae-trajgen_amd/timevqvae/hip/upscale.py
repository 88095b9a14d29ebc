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
from .conv import OP_DGRAD, OP_FWD, OP_WGRAD, PackCache, _conv_ws, _immediate, _keep
from .linear import gemm
from .xf import batch_colsum

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


# ------------------------------------------- Upscale's second conv folded into project_in
def hf_embed_supported(x, th, W_in, W2, pos_w):
    """x (B, H, m) = Upscale.first(tl), th (B, m, D), W_in (d, 2 D), W2 (D, H, 3)."""
    if not (x.is_cuda and x.dim() == 3 and th.dim() == 3 and W2.dim() == 3):
        return False
    B, H, m = x.shape
    D = th.shape[2]
    d = W_in.shape[0]
    return (th.shape[:2] == (B, m) and tuple(W2.shape) == (D, H, 3) and
            tuple(W_in.shape) == (d, 2 * D) and pos_w.shape[0] >= m and pos_w.shape[1] == 2 * D
            and d * (m + 1) <= 16384)


class _HFEmbedFolded(torch.autograd.Function):
    """project_in(cat(cls, cat(Conv1d(x, W2, b2)^T, th) + pos[:m])) without the (B, m + 1, 2 D)
    embedding or the 128-channel conv output (bidirectional_transformer.py:28-30,226-231 and
    x-transformers ContinuousTransformerWrapper.project_in, bias-free).  With W_in = [W_l | W_h]:
      v  = Conv1d(x, W_l W2) + W_l b2      (B, d, m): the conv computes d = 32 channels, not 128
      R  = th W_h^T (B m, d),  P = pos[:m] W_in^T (m, d),  Cp = cls W_in^T (B, d)
      z  = cat(Cp, v^T + R + P)            (tvq_hfe_assemble)
    Backward (dz -> dv, dR, dCp by tvq_hfe_assemble_bwd; dP = sum_b dR):
      dx = conv dgrad(dv, W_l W2);  G, s = conv wgrad / bias sum of (x, dv)
      dW2 = W_l^T G,  db2 = W_l^T s,  dth = dR W_h,  dcls = dCp W_in,  dpos[:m] += dP W_in
      dW_in = dCp^T cls + dP^T pos[:m] + [G W2^T + s b2^T | dR^T th]
    The same function as the unfolded chain up to fp32 reassociation."""

    @staticmethod
    def forward(ctx, x, th, cls_emb, W_in, W2, b2, pos_w):
        B, H, m = x.shape
        D = th.shape[2]
        d = W_in.shape[0]
        dev = x.device
        x4 = x.contiguous().view(B, H, 1, m)
        th2 = th.reshape(B * m, D).contiguous()
        cls2 = cls_emb.reshape(B, 2 * D).contiguous()
        W_in = W_in.contiguous()
        W2 = W2.contiguous()
        W_h = W_in[:, D:]
        W2c = gemm(W_in, 2 * D, 1, W2, 3 * H, 1, d, 3 * H, D)  # W_l W2 (d, H * 3)
        b2c = gemm(W_in, 2 * D, 1, b2, 1, 1, d, 1, D).view(d)
        v = torch.empty((B, d, 1, m), device=dev, dtype=torch.float32)
        ws = _conv_ws(OP_FWD, dev, B, H, 1, m, d, 1, 3, 1)
        with PackCache.paused():  # W2c is computed per call: never cached
            call("tvq_conv2d_fwd", ptr(x4), B, H, 1, m, ptr(W2c), ptr(b2c), d, 1, 3, 1, 0, ptr(v),
                 None, 0.0, None, 0, ptr(ws), stream_ptr())
        R = gemm(th2, D, 1, W_h, 1, 2 * D, B * m, d, D)
        P = gemm(pos_w, 2 * D, 1, W_in, 1, 2 * D, m, d, 2 * D)
        Cp = gemm(cls2, 2 * D, 1, W_in, 1, 2 * D, B, d, 2 * D)
        z = torch.empty((B, m + 1, d), device=dev, dtype=torch.float32)
        call("tvq_hfe_assemble", ptr(v), ptr(R), ptr(P), ptr(Cp), B, m, d, ptr(z), stream_ptr())
        ctx.save_for_backward(x4, th2, cls2, W_in, W2, b2, W2c)
        ctx.dims = (B, H, m, D, d, tuple(th.shape), tuple(cls_emb.shape))
        ctx.params = (W_in, W2, b2, pos_w)
        ctx.pos_w = pos_w
        return z

    @staticmethod
    def backward(ctx, gz):
        x4, th2, cls2, W_in, W2, b2, W2c = ctx.saved_tensors
        B, H, m, D, d, th_shape, cls_shape = ctx.dims
        dev = x4.device
        need = ctx.needs_input_grad
        g = gz.contiguous()
        dv = torch.empty((B, d, 1, m), device=dev, dtype=torch.float32)
        dR = torch.empty((B * m, d), device=dev, dtype=torch.float32)
        dCp = torch.empty((B, d), device=dev, dtype=torch.float32)
        call("tvq_hfe_assemble_bwd", ptr(g), B, m, d, ptr(dv), ptr(dR), ptr(dCp), stream_ptr())
        W_h = W_in[:, D:]
        dx = dth = dcls = None
        if need[0]:
            dx = torch.empty_like(x4)
            ws = _conv_ws(OP_DGRAD, dev, B, H, 1, m, d, 1, 3, 1)
            with PackCache.paused():
                call("tvq_conv2d_dgrad", ptr(dv), B, d, 1, m, ptr(W2c), H, 1, 3, 1, 0, ptr(dx), m,
                     ptr(ws), stream_ptr())
            dx = dx.view(B, H, m)
        if need[1]:
            dth = gemm(dR, d, 1, W_h, 2 * D, 1, B * m, D, d).view(th_shape)
        if need[2]:
            dcls = gemm(dCp, d, 1, W_in, 2 * D, 1, B, 2 * D, d).view(cls_shape)
        W_in_p, W2_p, b2_p, pos_p = ctx.params
        if not any(need[3:7]):
            return dx, dth, dcls, None, None, None, None
        sinks = [grad_sink(p) for p in ctx.params]
        direct = all(sk is not None for sk, nd in zip(sinks, need[3:7]) if nd)
        out = []
        for p, sk, nd in zip(ctx.params, sinks, need[3:7]):
            out.append((sk if direct else torch.zeros_like(p)) if nd else None)
        dWin, dW2, db2, dpos = out
        # weight gradients into the flat sinks are off the critical path (aux stream)
        with streams.offload(x4, dv, dR, dCp, th2, cls2) if direct else contextlib.nullcontext():
            G = torch.empty((d, H, 1, 3), device=dev, dtype=torch.float32)
            s = torch.empty(d, device=dev, dtype=torch.float32)
            ws = _conv_ws(OP_WGRAD, dev, B, H, 1, m, d, 1, 3, 1, required=True)
            with _immediate(True), PackCache.paused():
                call("tvq_conv2d_wgrad", ptr(x4), B, H, 1, m, ptr(dv), d, m, 1, 3, 1, 0, ptr(G),
                     ptr(s), 0, ptr(ws), stream_ptr())
            _keep(ws)
            dP = None
            if dWin is not None or dpos is not None:
                dP = torch.empty((m, d), device=dev, dtype=torch.float32)
                batch_colsum(dR.view(B, m, d), dP, d, False)
            if dWin is not None:
                L = 2 * D
                gemm(dCp, 1, d, cls2, L, 1, d, L, B, out=dWin, ldc=L, accumulate=True)
                gemm(dP, 1, d, ctx.pos_w, L, 1, d, L, m, out=dWin, ldc=L, accumulate=True)
                gemm(dR, 1, d, th2, D, 1, d, D, B * m, out=dWin[:, D:], ldc=L, accumulate=True)
                gemm(G, 3 * H, 1, W2, 1, 3 * H, d, D, 3 * H, out=dWin, ldc=L, accumulate=True)
                gemm(s, 1, 1, b2, 1, 1, d, D, 1, out=dWin, ldc=L, accumulate=True)
            if dW2 is not None:
                gemm(W_in, 1, 2 * D, G, 3 * H, 1, D, 3 * H, d, out=dW2, ldc=3 * H, accumulate=True)
            if db2 is not None:
                gemm(W_in, 1, 2 * D, s, 1, 1, D, 1, d, out=db2, ldc=1, accumulate=True)
            if dpos is not None:
                gemm(dP, d, 1, W_in, 2 * D, 1, m, 2 * D, d, out=dpos, ldc=2 * D, accumulate=True)
        if direct:
            return dx, dth, dcls, None, None, None, None
        return dx, dth, dcls, dWin, dW2, db2, dpos


def hf_embed_folded(x, th, cls_emb, W_in, W2, b2, pos_w):
    """z = project_in(cat(cls_emb, cat(Conv1d(x, W2, b2, padding=1)^T, th) + pos_w[:m])) for
    x (B, H, m), th (B, m, D), cls_emb (B, 1, 2 D) -> (B, m + 1, d), with autograd."""
    return _HFEmbedFolded.apply(x, th, cls_emb, W_in, W2, b2, pos_w)
