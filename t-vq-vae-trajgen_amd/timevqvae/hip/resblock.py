"""Fused ResBlock (include/tvq.h §fused ResBlock, csrc/tvq_resblock.hip, tvq_resblock_w8.hip).

ResBlock(C, C) of vq_vae.py:13-62 with C in {8, 16, 32} on the (B, C, 3, W) STFT image, and
C = 64 on the LF band's (B, 64, 3, 8) maps:
  y = x + Dropout_p(conv2(Snake_a2(BN(conv1(Snake_a1(x)) + b1))) + b2)
as 2 launches forward (training), 1 (eval), 2 backward, instead of one kernel per op.
`supported()` says when it applies; models/vq_vae.ResBlock falls back to the per-op path
otherwise (or when ENABLED is False: the tests' per-op comparison).
"""
import ctypes
import os

import torch

from . import rng
from ._native import call, grad_sink, ptr, stream_ptr, value
from .conv import _immediate, _keep

ENABLED = True


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


# ------------------------------------------------------- two consecutive ResBlocks
PAIR_ENABLED = True


def pair_supported(x):
    """Two consecutive identity ResBlocks on x's shape as one chain of 3 launches forward
    and 3 backward (rb_fwd1 | rb_fwd21 | rb_fwd2, rb_bwd2 | rb_bwd12 | rb_bwd1) instead of
    2 + 2 each: the middle launch runs block 1's second kernel and block 2's first on the
    same images, the activation handed over in registers; for the LF band's C = 64 blocks
    (tvq_resblock_w8.hip) w8_fwd21 / w8_bwd12 likewise, their BN finish launches between."""
    if not (ENABLED and PAIR_ENABLED) or x.dim() != 4 or not x.is_cuda:
        return False
    return bool(value("tvq_resblock_pair_supported", *x.shape))


def _arr(ts):
    return (ctypes.c_void_p * len(ts))(*[ptr(t) for t in ts])


class _ResBlockPairTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, *args):
        p1, p2 = args[0:8], args[8:16]
        rm1, rv1, nbt1, rm2, rv2, nbt2, momentum, eps, drop_p, site1, site2 = args[16:]
        x = x.contiguous()
        B, C, H, W = x.shape
        hs = value("tvq_resblock_saved_floats", B, C, H, W)
        h1 = torch.empty(hs, device=x.device)
        h2 = torch.empty(hs, device=x.device)
        y1 = torch.empty_like(x)
        y2 = torch.empty_like(x)
        save1 = torch.empty(4 * C, device=x.device)
        save2 = torch.empty(4 * C, device=x.device)
        seed = rng.seed_tensor(x.device) if drop_p > 0 else None
        # the offsets the two blocks draw in this order when run one by one
        off1 = rng.call_offset(site1) if drop_p > 0 else 0
        off2 = rng.call_offset(site2) if drop_p > 0 else 0
        keep = [_arr(p1), _arr(p2), _arr([rm1, rv1]), _arr([rm2, rv2])]
        ws1, ws2 = _ws(x), _ws(x)
        call("tvq_resblock_pair_train_fwd", ptr(x), B, C, H, W, *keep, ptr(nbt1), ptr(nbt2),
             float(momentum), float(eps), float(drop_p), ptr(seed), off1, off2, ptr(h1), ptr(y1),
             ptr(save1), ptr(h2), ptr(y2), ptr(save2), ptr(ws1), ptr(ws2), stream_ptr())
        ctx.save_for_backward(x, h1, y1, save1, h2, save2)
        ctx.params = (p1, p2)
        ctx.drop = (float(drop_p), off1, off2)
        ctx.seed = seed
        return y2

    @staticmethod
    def backward(ctx, gy):
        x, h1, y1, save1, h2, save2 = ctx.saved_tensors
        p1, p2 = ctx.params
        B, C, H, W = x.shape
        dev = x.device
        g = gy.contiguous()
        dx = torch.empty_like(x)
        dy1 = torch.empty_like(x)
        params = tuple(p1) + tuple(p2)
        has = [p is not None for p in params]
        sinks = [grad_sink(p) if p is not None else None for p in params]
        direct = all((s is not None) == hh for s, hh in zip(sinks, has))
        if direct:
            grads = sinks
        else:
            grads = [torch.empty(p.shape, device=dev) if p is not None else None for p in params]
        ws1, ws2 = _ws(x), _ws(x)
        drop_p, off1, off2 = ctx.drop

        def q(p, save):  # {a1, w1, bn_w, save, a2, w2}
            return _arr([p[0], p[1], p[3], save, p[5], p[6]])

        keep = [q(p1, save1), q(p2, save2), _arr(grads[0:8]), _arr(grads[8:16])]
        with _immediate(not direct):
            call("tvq_resblock_pair_bwd", ptr(g), ptr(x), B, C, H, W, keep[0], keep[1], ptr(h1),
                 ptr(y1), ptr(h2), drop_p, ptr(ctx.seed), off1, off2, ptr(dx), ptr(dy1), keep[2],
                 keep[3], int(direct), ptr(ws1), ptr(ws2), stream_ptr())
        _keep(ws1)
        _keep(ws2)
        out = [dx] + [None if direct else gr for gr in grads]
        return tuple(out) + (None,) * 11


def _block_args(rb):
    c = rb.convs
    return (c[0].a, c[1].weight, c[1].bias, c[2].weight, c[2].bias, c[3].a, c[4].weight,
            c[4].bias)


def resblock_pair_train(x, rb1, rb2, drop_p):
    """Training-mode fused pair of identity ResBlocks (models/vq_vae.ResBlock rb1, rb2 with
    equal BN momentum / eps and dropout p); bitwise equal to rb2(rb1(x)) on the fused path."""
    bn1, bn2 = rb1.convs[2], rb2.convs[2]
    if bn1.momentum is None or bn2.momentum is None:
        raise NotImplementedError("cumulative-average BatchNorm is not on the path")
    return _ResBlockPairTrain.apply(x, *_block_args(rb1), *_block_args(rb2), bn1.running_mean,
                                    bn1.running_var, bn1.num_batches_tracked, bn2.running_mean,
                                    bn2.running_var, bn2.num_batches_tracked, bn1.momentum,
                                    bn1.eps, float(drop_p), int(rb1._site), int(rb2._site))


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
