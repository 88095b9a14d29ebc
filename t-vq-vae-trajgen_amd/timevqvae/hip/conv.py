"""Convolutions on the HIP implicit-GEMM engine (include/tvq.h §convolutions).

conv2d          nn.Conv2d  (VQVAEEncBlock replicate 3x4 s(1,2); ResBlock 3x3; 1x1 proj;
                Conv1d k3 of Upscale as H=1) with fused bias / dropout / residual epilogue
conv_transpose2d nn.ConvTranspose2d 3x4 s(1,2) (VQVAEDecBlock, decoder tail)
Backward: dgrad (T/F gathers), wgrad (split positions, deterministic), bias = channel sum.
"""
import contextlib
import os

import torch

from . import rng, streams
from ._native import call, grad_sink, ptr, stream_ptr, value


def _ws(n, dev):
    return torch.empty(max(int(n), 1), device=dev, dtype=torch.float32)


def _bias_grad(g, dev, sink=None):
    """Per-channel sum of g (B, C, ...) -> returned tensor, or accumulated into `sink`."""
    B, C = g.shape[0], g.shape[1]
    HW = g.numel() // (B * C)
    out = sink if sink is not None else torch.empty(C, device=dev, dtype=torch.float32)
    ws = _ws(value("tvq_channel_sum_workspace", B, C, HW), dev)
    call("tvq_channel_sum", ptr(g), B, C, HW, ptr(out), int(sink is not None), ptr(ws),
         stream_ptr())
    return None if sink is not None else out


USE_WORKSPACE = True  # tests flip this to cover the no-workspace (in-place weight) path


_defer_keep = None  # workspaces of deferred weight-gradient reductions (wgrad_deferred)


DEFER_WGRAD = True  # False (tests): every weight-gradient split sum at once


@contextlib.contextmanager
def wgrad_deferred(this_stream_only=False):
    """Inside the scope the conv weight-gradient split sums are recorded and run by a few
    batched launches on the current stream at the exit (tvq_conv_wgrad_defer_*), bit for
    bit the same sums, instead of one reduction launch per conv.  Wrap a backward pass;
    gradients are final only after the exit.  this_stream_only: record only the reductions
    issued on the current stream -- conv weight gradients and the norm weight gradients
    accumulated into a flat gradient (a backward that runs on several streams); the others
    run at once."""
    global _defer_keep
    if _defer_keep is not None or not DEFER_WGRAD:
        yield  # nested (the outer scope flushes) or switched off
        return
    if this_stream_only:
        call("tvq_wgrad_defer_begin_stream", stream_ptr())
    else:
        call("tvq_conv_wgrad_defer_begin")
    _defer_keep = []
    try:
        yield
    finally:
        call("tvq_conv_wgrad_defer_flush", stream_ptr())
        _defer_keep = None  # freed after the flush is enqueued: stream-ordered reuse


def _keep(ws):
    if _defer_keep is not None and ws is not None:
        _defer_keep.append(ws)


@contextlib.contextmanager
def _immediate(needed_now):
    """A weight gradient returned to autograd (not written into a flat sink) is read right
    away: its reduction must not wait for the deferral scope's flush."""
    if needed_now and _defer_keep is not None:
        call("tvq_conv_wgrad_defer_pause", 1)
        try:
            yield
        finally:
            call("tvq_conv_wgrad_defer_pause", 0)
    else:
        yield


class PackCache:
    """Per-step weight-pack cache (include/tvq.h tvq_conv_packcache_*): inside `scope()` the
    staged-GEMM convs read [tap][c][n]-packed weights from one arena that the scope's entry
    repacks with a few batched launches, instead of one pack launch per conv call.  Open
    the scope around forward+backward only: the weights must not change inside it."""

    _next_id = [0]

    def __init__(self, device, floats=1 << 23):
        self.arena = torch.empty(int(floats), device=device, dtype=torch.float32)
        self.id = PackCache._next_id[0]
        PackCache._next_id[0] += 1

    @contextlib.contextmanager
    def scope(self):
        call("tvq_conv_packcache_begin", self.id, ptr(self.arena), self.arena.numel(),
             stream_ptr())
        try:
            yield self
        finally:
            call("tvq_conv_packcache_end")

    def __del__(self):
        try:
            call("tvq_conv_packcache_release", self.id)
        except Exception:  # interpreter shutdown: the library may be gone
            pass

    @staticmethod
    @contextlib.contextmanager
    def paused():
        """Convs inside bypass any open scope (for weights computed inside the scope: the
        cache repacks recorded weights at the next scope's begin, before such a weight is
        recomputed)."""
        call("tvq_conv_packcache_pause", 1)
        try:
            yield
        finally:
            call("tvq_conv_packcache_pause", 0)

    @staticmethod
    def entries():
        return value("tvq_conv_packcache_entries")

# tvq_conv_workspace ops
OP_FWD, OP_T_FWD, OP_DGRAD, OP_T_DGRAD, OP_WGRAD, OP_T_WGRAD = range(6)


def _conv_ws(op, dev, B, Ci, H, Wi, Co, KH, KW, SW, replicate=0, required=False):
    """Workspace for one conv op (weight repack + split-K partials [+ replicate canvas]);
    None for the optional forward-type workspaces when USE_WORKSPACE is off."""
    if not (USE_WORKSPACE or required):
        return None
    n = value("tvq_conv_workspace", op, B, Ci, H, Wi, Co, KH, KW, SW, int(replicate))
    return torch.empty(n, device=dev, dtype=torch.float32)


def _as4d(x):
    return x.unsqueeze(2) if x.dim() == 3 else x


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, SW, replicate, residual, drop_p, site):
        squeeze = x.dim() == 3
        x4 = _as4d(x).contiguous()
        w4 = _as4d(w).contiguous() if w.dim() == 3 else w.contiguous()
        B, Ci, H, Wi = x4.shape
        Co, _, KH, KW = w4.shape
        Wo = value("tvq_conv_out_width", Wi, KW, SW, 0)
        y = torch.empty((B, Co, H, Wo), device=x.device, dtype=torch.float32)
        res = _as4d(residual).contiguous() if residual is not None else None
        seed = rng.seed_tensor(x.device) if drop_p > 0 else None
        off = rng.call_offset(site) if drop_p > 0 else 0
        ws = _conv_ws(OP_FWD, x.device, B, Ci, H, Wi, Co, KH, KW, SW)
        call("tvq_conv2d_fwd", ptr(x4), B, Ci, H, Wi, ptr(w4), ptr(b), Co, KH, KW, SW,
             int(replicate), ptr(y), ptr(res), float(drop_p), ptr(seed), off, ptr(ws),
             stream_ptr())
        ctx.save_for_backward(x4, w4)
        ctx.cfg = (SW, replicate, drop_p, off, squeeze, b is not None, residual is not None,
                   w.dim())
        ctx.seed = seed
        ctx.params = (w, b)
        return y.squeeze(2) if squeeze else y

    @staticmethod
    def backward(ctx, gy):
        x4, w4 = ctx.saved_tensors
        SW, replicate, drop_p, off, squeeze, has_b, has_res, wdim = ctx.cfg
        B, Ci, H, Wi = x4.shape
        Co, _, KH, KW = w4.shape
        dev = x4.device
        s = stream_ptr()
        g = _as4d(gy).contiguous()
        Wo = g.shape[3]
        if drop_p > 0:
            gd = torch.empty_like(g)
            call("tvq_dropout_bwd", ptr(g), g.numel(), float(drop_p), ptr(ctx.seed), off, ptr(gd), s)
        else:
            gd = g
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x4)
            ws = _conv_ws(OP_DGRAD, dev, B, Ci, H, Wi, Co, KH, KW, SW, replicate,
                          required=bool(replicate))
            call("tvq_conv2d_dgrad", ptr(gd), B, Co, H, Wo, ptr(w4), Ci, KH, KW, SW,
                 int(replicate), ptr(dx), Wi, ptr(ws), s)
            if squeeze:
                dx = dx.squeeze(2)
        need_w, need_b = ctx.needs_input_grad[1], has_b and ctx.needs_input_grad[2]
        if need_w or need_b:
            w_p, b_p = ctx.params
            sw, sb = grad_sink(w_p), grad_sink(b_p) if has_b else None
            direct = need_w and sw is not None and (not need_b or sb is not None)
            # gradients into the flat sinks are off the critical path: aux stream
            with (streams.offload(x4, gd) if direct else contextlib.nullcontext()):
                dwt = sw if direct else torch.empty_like(w4)
                dbt = (sb if direct else torch.empty(Co, device=dev)) if need_b else None
                ws = _conv_ws(OP_WGRAD, dev, B, Ci, H, Wi, Co, KH, KW, SW, replicate,
                              required=True)
                with _immediate(not direct):
                    call("tvq_conv2d_wgrad", ptr(x4), B, Ci, H, Wi, ptr(gd), Co, Wo, KH, KW, SW,
                         int(replicate), ptr(dwt), ptr(dbt), int(direct), ptr(ws), stream_ptr())
                _keep(ws)
            if not direct:
                dw = (dwt.squeeze(2) if wdim == 3 else dwt) if need_w else None
                db = dbt
        dres = None
        if has_res and ctx.needs_input_grad[5]:
            dres = gy
        return dx, dw, db, None, None, dres, None, None


def conv2d(x, weight, bias=None, stride_w=1, replicate=False, residual=None, drop_p=0.0, site=0):
    """y = residual + Dropout_p(conv(x) + bias).  x (B,C,H,W) or (B,C,L) with a (Co,Ci,KH,KW) /
    (Co,Ci,K) weight; padding (KH//2, (KW-1)//2), zero or replicate."""
    return _Conv2d.apply(x, weight, bias, int(stride_w), bool(replicate), residual, float(drop_p),
                         int(site))


class _ConvT2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, SW):
        x = x.contiguous()
        w = w.contiguous()
        B, Ci, H, Wi = x.shape
        _, Co, KH, KW = w.shape
        Wo = value("tvq_conv_out_width", Wi, KW, SW, 1)
        y = torch.empty((B, Co, H, Wo), device=x.device, dtype=torch.float32)
        ws = _conv_ws(OP_T_FWD, x.device, B, Ci, H, Wi, Co, KH, KW, SW)
        call("tvq_convT2d_fwd", ptr(x), B, Ci, H, Wi, ptr(w), ptr(b), Co, KH, KW, SW, ptr(y), None,
             ptr(ws), stream_ptr())
        ctx.save_for_backward(x, w)
        ctx.SW = SW
        ctx.has_b = b is not None
        ctx.params = (w, b)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        SW = ctx.SW
        B, Ci, H, Wi = x.shape
        _, Co, KH, KW = w.shape
        g = gy.contiguous()
        Wo = g.shape[3]
        s = stream_ptr()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            ws = _conv_ws(OP_T_DGRAD, x.device, B, Ci, H, Wi, Co, KH, KW, SW)
            call("tvq_convT2d_dgrad", ptr(g), B, Co, H, Wo, ptr(w), Ci, KH, KW, SW, ptr(dx), Wi,
                 ptr(ws), s)
        w_p, b_p = ctx.params
        if ctx.needs_input_grad[1]:
            sw = grad_sink(w_p)
            with (streams.offload(x, g) if sw is not None else contextlib.nullcontext()):
                dwt = sw if sw is not None else torch.empty_like(w)
                ws = _conv_ws(OP_T_WGRAD, x.device, B, Ci, H, Wi, Co, KH, KW, SW, required=True)
                with _immediate(sw is None):
                    call("tvq_convT2d_wgrad", ptr(x), B, Ci, H, Wi, ptr(g), Co, Wo, KH, KW, SW,
                         ptr(dwt), int(sw is not None), ptr(ws), stream_ptr())
                _keep(ws)
            dw = None if sw is not None else dwt
        if ctx.has_b and ctx.needs_input_grad[2]:
            sb = grad_sink(b_p)
            with (streams.offload(g) if sb is not None else contextlib.nullcontext()):
                db = _bias_grad(g, x.device, sb)
        return dx, dw, db, None


def conv_transpose2d(x, weight, bias=None, stride_w=2):
    return _ConvT2d.apply(x, weight, bias, int(stride_w))


def bnstats_blocks(x, weight, stride_w, transposed):
    """Per-channel partials tvq_conv2d_fwd_bnstats writes for this conv (0: the shape does not
    take the stride-2 kernels; the conv and its BatchNorm then run apart)."""
    if x.dim() != 4 or weight.dim() != 4:
        return 0
    B, Ci, H, Wi = x.shape
    Co = weight.shape[1] if transposed else weight.shape[0]
    KH, KW = weight.shape[2], weight.shape[3]
    return int(value("tvq_conv_bnstats_blocks", B, Ci, H, Wi, Co, KH, KW, int(stride_w),
                     int(bool(transposed))))


def _bnstats_fwd(ctx, x, w, b, SW, replicate, transposed):
    x = x.contiguous()
    w = w.contiguous()
    B, Ci, H, Wi = x.shape
    Co = w.shape[1] if transposed else w.shape[0]
    KH, KW = w.shape[2], w.shape[3]
    Wo = value("tvq_conv_out_width", Wi, KW, SW, int(bool(transposed)))
    nblk = value("tvq_conv_bnstats_blocks", B, Ci, H, Wi, Co, KH, KW, SW, int(bool(transposed)))
    y = torch.empty((B, Co, H, Wo), device=x.device, dtype=torch.float32)
    part = torch.empty((Co, nblk, 2), device=x.device, dtype=torch.float64)
    call("tvq_conv2d_fwd_bnstats", ptr(x), B, Ci, H, Wi, ptr(w), ptr(b), Co, KH, KW, SW,
         int(bool(replicate)), int(bool(transposed)), ptr(y), ptr(part), stream_ptr())
    ctx.mark_non_differentiable(part)
    ctx.set_materialize_grads(False)  # no zero-filled gradient for `part` (an aten fill)
    return x, w, y, part


class _Conv2dStats(_Conv2d):
    """conv2d (stride-2 EncBlock conv) that also returns its output's per-block BatchNorm
    statistics (tvq_conv2d_fwd_bnstats); backward = _Conv2d's."""

    @staticmethod
    def forward(ctx, x, w, b, SW, replicate):
        x4, w4, y, part = _bnstats_fwd(ctx, x, w, b, SW, replicate, False)
        ctx.save_for_backward(x4, w4)
        ctx.cfg = (SW, replicate, 0.0, 0, False, b is not None, False, 4)
        ctx.seed = None
        ctx.params = (w, b)
        return y, part

    @staticmethod
    def backward(ctx, gy, gpart):
        return _Conv2d.backward(ctx, gy)[:5]


class _ConvT2dStats(_ConvT2d):
    """conv_transpose2d (stride-2 DecBlock conv) + per-block BatchNorm statistics."""

    @staticmethod
    def forward(ctx, x, w, b, SW):
        x4, w4, y, part = _bnstats_fwd(ctx, x, w, b, SW, False, True)
        ctx.save_for_backward(x4, w4)
        ctx.SW = SW
        ctx.has_b = b is not None
        ctx.params = (w, b)
        return y, part

    @staticmethod
    def backward(ctx, gy, gpart):
        return _ConvT2d.backward(ctx, gy)


def conv2d_bnstats(x, weight, bias, stride_w=2, replicate=False):
    """(conv2d(x), per-block BatchNorm statistics of it) for bn_snake_part; the caller checks
    bnstats_blocks(x, weight, stride_w, False) > 0 first."""
    return _Conv2dStats.apply(x, weight, bias, int(stride_w), bool(replicate))


def conv_transpose2d_bnstats(x, weight, bias, stride_w=2):
    return _ConvT2dStats.apply(x, weight, bias, int(stride_w))


FUSED_BN_EVAL = True  # False (tests): the eval conv and BN as separate launches


def bn_eval_fusable(x, bn, *params):
    """An eval-mode conv -> BN (-> Snake) pair can run as one launch when nothing needs a
    gradient (the sampler's decoders, vq_vae.py:31-48,98-118)."""
    if not FUSED_BN_EVAL or bn.training:
        return False
    if torch.is_grad_enabled() and (x.requires_grad or any(
            p is not None and p.requires_grad for p in params + (bn.weight, bn.bias))):
        return False
    return True


def conv2d_bn_eval(x, weight, bias, bn, a=None, stride_w=1, replicate=False, pre_gelu=False):
    """snake_a(BatchNorm_eval([GELU](conv(x) + bias))) in one launch (tvq_conv2d_fwd_bn_eval);
    no autograd.  a: the Snake parameter or None."""
    squeeze = x.dim() == 3
    x4 = _as4d(x).contiguous()
    w4 = _as4d(weight).contiguous() if weight.dim() == 3 else weight.contiguous()
    B, Ci, H, Wi = x4.shape
    Co, _, KH, KW = w4.shape
    SW = int(stride_w)
    Wo = value("tvq_conv_out_width", Wi, KW, SW, 0)
    y = torch.empty((B, Co, H, Wo), device=x.device, dtype=torch.float32)
    ws = _conv_ws(OP_FWD, x.device, B, Ci, H, Wi, Co, KH, KW, SW)
    call("tvq_conv2d_fwd_bn_eval", ptr(x4), B, Ci, H, Wi, ptr(w4), ptr(bias), Co, KH, KW, SW,
         int(replicate), int(pre_gelu), ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean),
         ptr(bn.running_var),
         float(bn.eps), ptr(a.reshape(-1) if a is not None else None), ptr(y), ptr(ws),
         stream_ptr())
    return y.squeeze(2) if squeeze else y


def conv_transpose2d_bn_eval(x, weight, bias, bn, a=None, stride_w=2):
    """snake_a(BatchNorm_eval(conv_transpose(x) + bias)) in one launch; no autograd."""
    x = x.contiguous()
    w = weight.contiguous()
    B, Ci, H, Wi = x.shape
    _, Co, KH, KW = w.shape
    SW = int(stride_w)
    Wo = value("tvq_conv_out_width", Wi, KW, SW, 1)
    y = torch.empty((B, Co, H, Wo), device=x.device, dtype=torch.float32)
    ws = _conv_ws(OP_T_FWD, x.device, B, Ci, H, Wi, Co, KH, KW, SW)
    call("tvq_convT2d_fwd_bn_eval", ptr(x), B, Ci, H, Wi, ptr(w), ptr(bias), Co, KH, KW, SW,
         ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean), ptr(bn.running_var), float(bn.eps),
         ptr(a.reshape(-1) if a is not None else None), ptr(y), ptr(ws), stream_ptr())
    return y
