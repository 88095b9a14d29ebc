"""Fused ResBlock (include/tvq.h §fused ResBlock, csrc/tvq_resblock.hip, tvq_resblock_w8.hip).

ResBlock(C, C) of vq_vae.py:13-62 with C in {8, 16, 32} on the (B, C, 3, W) STFT image, and
C = 64 on the LF band's (B, 64, 3, 8) maps:
  y = x + Dropout_p(conv2(Snake_a2(BN(conv1(Snake_a1(x)) + b1))) + b2)
as 2 launches forward (training), 1 (eval), 2 backward, instead of one kernel per op.
`supported()` says when it applies; models/vq_vae.ResBlock falls back to the per-op path
otherwise (or when TVQ_RESBLOCK_FUSED=0).
"""
import os

import torch

from . import rng
from ._native import call, grad_sink, ptr, stream_ptr, value
from .conv import _immediate, _keep

ENABLED = os.environ.get("TVQ_RESBLOCK_FUSED", "1") != "0"


def supported(x, C_in, C_out):
    if not ENABLED or C_in != C_out or x.dim() != 4 or not x.is_cuda:
        return False
    B, C, H, W = x.shape
    return C == C_in and value("tvq_resblock_workspace", B, C, H, W) > 0


def _ws(x):
    B, C, H, W = x.shape
    return torch.empty(value("tvq_resblock_workspace", B, C, H, W), device=x.device,
                       dtype=torch.uint8)


class _ResBlockTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, a1, w1, b1, bn_w, bn_b, a2, w2, b2, rmean, rvar, nbt, momentum, eps,
                drop_p, site):
        x = x.contiguous()
        B, C, H, W = x.shape
        # the backward's saved activations: conv1's output (and, C = 64, the two Snake
        # outputs the weight gradients read)
        h = torch.empty(value("tvq_resblock_saved_floats", B, C, H, W), device=x.device)
        y = torch.empty_like(x)
        save = torch.empty(4 * C, device=x.device, dtype=torch.float32)
        seed = rng.seed_tensor(x.device) if drop_p > 0 else None
        off = rng.call_offset(site) if drop_p > 0 else 0
        call("tvq_resblock_train_fwd", ptr(x), B, C, H, W, ptr(a1), ptr(w1), ptr(b1), ptr(bn_w),
             ptr(bn_b), ptr(rmean), ptr(rvar), ptr(nbt), float(momentum), float(eps), ptr(a2),
             ptr(w2), ptr(b2), float(drop_p), ptr(seed), off, ptr(h), ptr(y), ptr(save),
             ptr(_ws(x)), stream_ptr())
        ctx.save_for_backward(x, h, save)
        ctx.params = (a1, w1, b1, bn_w, bn_b, a2, w2, b2)
        ctx.drop = (float(drop_p), off)
        ctx.seed = seed
        return y

    @staticmethod
    def backward(ctx, gy):
        x, h, save = ctx.saved_tensors
        a1, w1, b1, bn_w, bn_b, a2, w2, b2 = ctx.params
        B, C, H, W = x.shape
        dev = x.device
        g = gy.contiguous()
        dx = torch.empty_like(x)
        params = ctx.params
        has = [p is not None for p in params]
        sinks = [grad_sink(p) if p is not None else None for p in params]
        direct = all((s is not None) == hh for s, hh in zip(sinks, has))
        if direct:
            grads = sinks
        else:
            grads = [torch.empty(p.shape, device=dev) if p is not None else None for p in params]
        da1, dw1, db1, dbw, dbb, da2, dw2, db2 = grads
        ws = _ws(x)
        drop_p, off = ctx.drop
        with _immediate(not direct):
            call("tvq_resblock_bwd", ptr(g), ptr(x), ptr(h), B, C, H, W, ptr(a1), ptr(w1),
                 ptr(bn_w), ptr(save), ptr(a2), ptr(w2), drop_p, ptr(ctx.seed), off, ptr(dx),
                 ptr(da1), ptr(dw1), ptr(db1), ptr(dbw), ptr(dbb), ptr(da2), ptr(dw2), ptr(db2),
                 int(direct), ptr(ws), stream_ptr())
        _keep(ws)
        out = [dx] + [None if direct else gr for gr in grads]
        return tuple(out) + (None,) * 7


def resblock_train(x, a1, conv1, bn, a2, conv2, drop_p, site):
    """Training-mode fused ResBlock; a1/a2: the Snake (1,C,1,1) parameters."""
    if bn.momentum is None:
        raise NotImplementedError("cumulative-average BatchNorm is not on the path")
    return _ResBlockTrain.apply(x, a1, conv1.weight, conv1.bias, bn.weight, bn.bias, a2,
                                conv2.weight, conv2.bias, bn.running_mean, bn.running_var,
                                bn.num_batches_tracked, bn.momentum, bn.eps, float(drop_p),
                                int(site))


def resblock_eval(x, a1, conv1, bn, a2, conv2):
    """Eval-mode fused ResBlock (BN from the running statistics), no autograd."""
    x = x.contiguous()
    B, C, H, W = x.shape
    y = torch.empty_like(x)
    call("tvq_resblock_eval_fwd", ptr(x), B, C, H, W, ptr(a1), ptr(conv1.weight), ptr(conv1.bias),
         ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean), ptr(bn.running_var), float(bn.eps),
         ptr(a2), ptr(conv2.weight), ptr(conv2.bias), ptr(y), stream_ptr())
    return y


# ---------------------------------------------------------------- projection ResBlock
def proj_supported(x, C_in, C_out):
    """ResBlock(C_in, C_out) with the 1x1 projection on the skip, on the LF band's W = 8
    maps: 64 -> 128 (the encoder's last block) and 128 -> 64 (the decoder's first)
    (csrc/tvq_resblock_w8p.hip)."""
    if not ENABLED or C_in == C_out or x.dim() != 4 or not x.is_cuda:
        return False
    B, C, H, W = x.shape
    return C == C_in and value("tvq_resblock_proj_workspace", B, C_in, C_out, H, W) > 0


def _pws(x, Co):
    B, C, H, W = x.shape
    return torch.empty(value("tvq_resblock_proj_workspace", B, C, Co, H, W), device=x.device,
                       dtype=torch.uint8)


class _ResBlockProjTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, a1, w1, b1, bn_w, bn_b, a2, w2, b2, wp, bp, rmean, rvar, nbt, momentum,
                eps, drop_p, site):
        x = x.contiguous()
        B, Ci, H, W = x.shape
        Co = w1.shape[0]
        h = torch.empty(value("tvq_resblock_proj_saved_floats", B, Ci, Co, H, W), device=x.device)
        y = torch.empty((B, Co, H, W), device=x.device)
        save = torch.empty(4 * Co, device=x.device, dtype=torch.float32)
        seed = rng.seed_tensor(x.device) if drop_p > 0 else None
        off = rng.call_offset(site) if drop_p > 0 else 0
        call("tvq_resblock_proj_train_fwd", ptr(x), B, Ci, Co, H, W, ptr(a1), ptr(w1), ptr(b1),
             ptr(bn_w), ptr(bn_b), ptr(rmean), ptr(rvar), ptr(nbt), float(momentum), float(eps),
             ptr(a2), ptr(w2), ptr(b2), ptr(wp), ptr(bp), float(drop_p), ptr(seed), off, ptr(h),
             ptr(y), ptr(save), ptr(_pws(x, Co)), stream_ptr())
        ctx.save_for_backward(x, h, save)
        ctx.params = (a1, w1, b1, bn_w, bn_b, a2, w2, b2, wp, bp)
        ctx.drop = (float(drop_p), off)
        ctx.seed = seed
        return y

    @staticmethod
    def backward(ctx, gy):
        x, h, save = ctx.saved_tensors
        a1, w1, b1, bn_w, bn_b, a2, w2, b2, wp, bp = ctx.params
        B, Ci, H, W = x.shape
        Co = w1.shape[0]
        dev = x.device
        g = gy.contiguous()
        dx = torch.empty_like(x)
        params = ctx.params
        has = [p is not None for p in params]
        sinks = [grad_sink(p) if p is not None else None for p in params]
        direct = all((s is not None) == hh for s, hh in zip(sinks, has))
        if direct:
            grads = sinks
        else:
            grads = [torch.empty(p.shape, device=dev) if p is not None else None for p in params]
        da1, dw1, db1, dbw, dbb, da2, dw2, db2, dwp, dbp = grads
        ws = _pws(x, Co)
        drop_p, off = ctx.drop
        with _immediate(not direct):
            call("tvq_resblock_proj_bwd", ptr(g), ptr(x), ptr(h), B, Ci, Co, H, W, ptr(a1),
                 ptr(w1), ptr(bn_w), ptr(save), ptr(a2), ptr(w2), ptr(wp), drop_p, ptr(ctx.seed),
                 off, ptr(dx), ptr(da1), ptr(dw1), ptr(db1), ptr(dbw), ptr(dbb), ptr(da2), ptr(dw2),
                 ptr(db2), ptr(dwp), ptr(dbp), int(direct), ptr(ws), stream_ptr())
        _keep(ws)
        out = [dx] + [None if direct else gr for gr in grads]
        return tuple(out) + (None,) * 7


def resblock_proj_train(x, a1, conv1, bn, a2, conv2, proj, drop_p, site):
    """Training-mode fused projection ResBlock; a1/a2: the Snake (1,C,1,1) parameters."""
    if bn.momentum is None:
        raise NotImplementedError("cumulative-average BatchNorm is not on the path")
    return _ResBlockProjTrain.apply(x, a1, conv1.weight, conv1.bias, bn.weight, bn.bias, a2,
                                    conv2.weight, conv2.bias, proj.weight, proj.bias,
                                    bn.running_mean, bn.running_var, bn.num_batches_tracked,
                                    bn.momentum, bn.eps, float(drop_p), int(site))


def resblock_proj_eval(x, a1, conv1, bn, a2, conv2, proj):
    """Eval-mode fused projection ResBlock (BN from the running statistics), no autograd."""
    x = x.contiguous()
    B, Ci, H, W = x.shape
    Co = conv1.weight.shape[0]
    y = torch.empty((B, Co, H, W), device=x.device)
    call("tvq_resblock_proj_eval_fwd", ptr(x), B, Ci, Co, H, W, ptr(a1), ptr(conv1.weight),
         ptr(conv1.bias), ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean),
         ptr(bn.running_var), float(bn.eps), ptr(a2), ptr(conv2.weight), ptr(conv2.bias),
         ptr(proj.weight), ptr(proj.bias), ptr(y), stream_ptr())
    return y
