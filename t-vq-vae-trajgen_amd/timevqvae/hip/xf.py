"""MaskGIT transformer ops on the HIP path (include/tvq.h §MaskGIT transformer)."""
import contextlib
import math
import os

import torch

from . import rng, streams, wgrad
from ._native import call, grad_sink, ptr, stream_ptr, value
from .conv import _keep
from .linear import _bias_grad_rows, gemm, weight_grad


def _rows(x):
    D = x.shape[-1]
    return x.reshape(-1, D), x.numel() // D, D


# ------------------------------------------------------------------ RMSNorm
class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, scale):
        x2, M, D = _rows(x.contiguous())
        y = torch.empty_like(x2)
        inv = torch.empty(M, device=x.device, dtype=torch.float32)
        call("tvq_rmsnorm_fwd", ptr(x2), M, D, ptr(g), float(scale), ptr(y), ptr(inv), stream_ptr())
        ctx.save_for_backward(x2, g, inv)
        ctx.g_param = g
        ctx.scale = scale
        ctx.shape = x.shape
        return y.reshape(x.shape)

    @staticmethod
    def backward(ctx, gy):
        x2, g, inv = ctx.saved_tensors
        M, D = x2.shape
        dy = gy.reshape(M, D).contiguous()
        dx = torch.empty_like(x2)
        sink = grad_sink(ctx.g_param)
        dg = sink if sink is not None else torch.empty(D, device=x2.device)
        ws = torch.empty(value("tvq_norm_bwd_workspace", M, D), device=x2.device)
        call("tvq_rmsnorm_bwd", ptr(dy), ptr(x2), M, D, ptr(g), float(ctx.scale), ptr(inv), None,
             ptr(dx), ptr(dg), int(sink is not None), ptr(ws), stream_ptr())
        _keep(ws)  # its reduction may be deferred (hip.conv.wgrad_deferred)
        return dx.reshape(ctx.shape), (None if sink is not None else dg), None


def rmsnorm(x, g):
    """x-transformers RMSNorm: F.normalize(x, dim=-1) * sqrt(D) * g."""
    return _RMSNorm.apply(x, g, math.sqrt(x.shape[-1]))


class _RMSNormRes(torch.autograd.Function):
    """(RMSNorm(x), x) for a pre-norm residual layer x + f(RMSNorm(x)): the second output
    (the residual stream) is what the branch's output Linear adds, so x has a single
    autograd consumer and dx = RMSNorm'(dn) + dres comes out of one kernel instead of an
    autograd accumulation add."""

    @staticmethod
    def forward(ctx, x, g, scale):
        x2, M, D = _rows(x.contiguous())
        y = torch.empty_like(x2)
        inv = torch.empty(M, device=x.device, dtype=torch.float32)
        call("tvq_rmsnorm_fwd", ptr(x2), M, D, ptr(g), float(scale), ptr(y), ptr(inv), stream_ptr())
        ctx.save_for_backward(x2, g, inv)
        ctx.g_param = g
        ctx.scale = scale
        ctx.shape = x.shape
        return y.reshape(x.shape), x.view_as(x)

    @staticmethod
    def backward(ctx, gy, gr):
        x2, g, inv = ctx.saved_tensors
        M, D = x2.shape
        dx = torch.empty_like(x2)
        if gy is None:  # the normalised output unused: only the residual path
            return gr, None, None
        dy = gy.reshape(M, D).contiguous()
        dres = gr.reshape(M, D).contiguous() if gr is not None else None
        sink = grad_sink(ctx.g_param)
        dg = sink if sink is not None else torch.empty(D, device=x2.device)
        ws = torch.empty(value("tvq_norm_bwd_workspace", M, D), device=x2.device)
        call("tvq_rmsnorm_bwd", ptr(dy), ptr(x2), M, D, ptr(g), float(ctx.scale), ptr(inv),
             ptr(dres), ptr(dx), ptr(dg), int(sink is not None), ptr(ws), stream_ptr())
        _keep(ws)
        return dx.reshape(ctx.shape), (None if sink is not None else dg), None


def rmsnorm_res(x, g):
    """(RMSNorm(x), residual stream x) with the residual gradient summed in the norm's
    backward kernel (see _RMSNormRes)."""
    return _RMSNormRes.apply(x, g, math.sqrt(x.shape[-1]))


# ---------------------------------------------------------------- LayerNorm
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        x2, M, D = _rows(x.contiguous())
        y = torch.empty_like(x2)
        mean = torch.empty(M, device=x.device)
        rstd = torch.empty(M, device=x.device)
        call("tvq_layernorm_fwd", ptr(x2), M, D, ptr(gamma), ptr(beta), float(eps), ptr(y),
             ptr(mean), ptr(rstd), stream_ptr())
        ctx.save_for_backward(x2, gamma, mean, rstd)
        ctx.params = (gamma, beta)
        ctx.has = (gamma is not None, beta is not None)
        ctx.shape = x.shape
        return y.reshape(x.shape)

    @staticmethod
    def backward(ctx, gy):
        x2, gamma, mean, rstd = ctx.saved_tensors
        M, D = x2.shape
        dy = gy.reshape(M, D).contiguous()
        dx = torch.empty_like(x2)
        sinks = [grad_sink(p) if h else None for p, h in zip(ctx.params, ctx.has)]
        direct = all((s is not None) == h for s, h in zip(sinks, ctx.has))
        if direct:
            dg, db = sinks
        else:
            dg = torch.empty(D, device=x2.device) if ctx.has[0] else None
            db = torch.empty(D, device=x2.device) if ctx.has[1] else None
        ws = torch.empty(value("tvq_norm_bwd_workspace", M, D), device=x2.device)
        call("tvq_layernorm_bwd", ptr(dy), ptr(x2), M, D, ptr(gamma), ptr(mean), ptr(rstd), ptr(dx),
             ptr(dg), ptr(db), int(direct), ptr(ws), stream_ptr())
        _keep(ws)
        if direct:
            return dx.reshape(ctx.shape), None, None, None
        return dx.reshape(ctx.shape), dg, db, None


def layer_norm(x, gamma=None, beta=None, eps=1e-5):
    return _LayerNorm.apply(x, gamma, beta, float(eps))


# ---------------------------------------------------------------- Linear (+GELU)
class _LinearAct(torch.autograd.Function):
    """y = act(x W^T + b); act 1 = GELU(erf) with the pre-activation kept for backward."""

    @staticmethod
    def forward(ctx, x, w, b, act):
        K = x.shape[-1]
        N = w.shape[0]
        x2 = x.reshape(-1, K).contiguous()
        w = w.contiguous()
        M = x2.shape[0]
        pre = torch.empty((M, N), device=x.device) if act else None
        y = gemm(x2, K, 1, w, 1, K, M, N, K, bias=b, act=act, pre=pre)
        ctx.save_for_backward(x2, w, pre)
        ctx.params = (w, b)
        ctx.wg_tag = wgrad.current_tag()
        ctx.act = act
        ctx.has_b = b is not None
        ctx.shape = x.shape
        return y.reshape(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, gy):
        x2, w, pre = ctx.saved_tensors
        M, K = x2.shape
        N = w.shape[0]
        g = gy.reshape(M, N).contiguous()
        if ctx.act:
            gp = torch.empty_like(g)
            call("tvq_gelu_bwd", ptr(g), ptr(pre), g.numel(), ptr(gp), stream_ptr())
            g = gp
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = gemm(g, N, 1, w, K, 1, M, K, N).reshape(ctx.shape)
        if ctx.needs_input_grad[1] and ctx.has_b and ctx.needs_input_grad[2]:
            dw, db = weight_grad(g, x2, ctx.params[0], M, N, K, ctx.wg_tag, ctx.params[1])
        else:
            if ctx.needs_input_grad[1]:
                dw = weight_grad(g, x2, ctx.params[0], M, N, K, ctx.wg_tag)
            if ctx.has_b and ctx.needs_input_grad[2]:
                db = _bias_grad_rows(g, grad_sink(ctx.params[1]))
        return dx, dw, db, None


def linear_act(x, weight, bias=None, gelu=False):
    return _LinearAct.apply(x, weight, bias, 1 if gelu else 0)


# ---------------------------------------------------------------- fused feed-forward
FUSED_FF = True


class _FusedFF(torch.autograd.Function):
    """r + gate * (dropout(GELU(xn W1^T + b1)) W2^T + b2) with D = inner = 128 in one launch
    forward and one backward (csrc/tvq_ffn.hip; x-transformers FeedForward in the pre-norm
    residual, bidirectional_transformer.py:92-110).  Weight / bias gradients go through the
    grouped weight-gradient path like every Linear's; dW2 / db2 are taken from gate * gy,
    which the backward kernel writes when a gate is given (as the per-op path's scale_by):
    a forward whose branch was dropped adds exactly zero to them, whatever other forwards
    (gradient accumulation) or replicas did with the same segment."""

    @staticmethod
    def forward(ctx, xn, r, w1, b1, w2, b2, gate, p, site):
        shp = xn.shape
        x2 = xn.reshape(-1, 128).contiguous()
        r2 = r.reshape(-1, 128).contiguous()
        M = x2.shape[0]
        y, pre, hd = (torch.empty_like(x2) for _ in range(3))
        seed = rng.seed_tensor(xn.device) if p > 0 else None
        off = rng.call_offset(site) if p > 0 else 0
        call("tvq_ffn_fwd", ptr(x2), ptr(r2), M, 128, ptr(w1), ptr(b1), ptr(w2), ptr(b2),
             ptr(gate), float(p), ptr(seed), off, ptr(y), ptr(pre), ptr(hd), stream_ptr())
        ctx.save_for_backward(x2, pre, hd, w1, w2)
        ctx.cfg = (float(p), off, shp)
        ctx.seed, ctx.gate = seed, gate
        ctx.params = (w1, b1, w2, b2)
        ctx.wg_tag = wgrad.current_tag()
        return y.reshape(shp)

    @staticmethod
    def backward(ctx, gy):
        x2, pre, hd, w1, w2 = ctx.saved_tensors
        p, off, shp = ctx.cfg
        g2 = gy.reshape(-1, 128).contiguous()
        M = g2.shape[0]
        d_pre, dxn = torch.empty_like(g2), torch.empty_like(g2)
        need = ctx.needs_input_grad
        gg = torch.empty_like(g2) if ctx.gate is not None and (need[4] or need[5]) else None
        call("tvq_ffn_bwd", ptr(g2), ptr(pre), M, 128, ptr(w1), ptr(w2), ptr(ctx.gate), p,
             ptr(ctx.seed), off, ptr(d_pre), ptr(dxn), ptr(gg), stream_ptr())
        W1p, b1p, W2p, b2p = ctx.params
        g2w = gg if gg is not None else g2
        dw1 = db1 = dw2 = db2 = None
        if need[4] and need[5]:  # weight and bias gradients in one grouped record
            dw2, db2 = weight_grad(g2w, hd, W2p, M, 128, 128, ctx.wg_tag, b2p)
        else:
            dw2 = weight_grad(g2w, hd, W2p, M, 128, 128, ctx.wg_tag) if need[4] else None
            db2 = _bias_grad_rows(g2w, grad_sink(b2p)) if need[5] else None
        if need[2] and need[3]:
            dw1, db1 = weight_grad(d_pre, x2, W1p, M, 128, 128, ctx.wg_tag, b1p)
        else:
            dw1 = weight_grad(d_pre, x2, W1p, M, 128, 128, ctx.wg_tag) if need[2] else None
            db1 = _bias_grad_rows(d_pre, grad_sink(b1p)) if need[3] else None
        return (dxn.reshape(shp) if need[0] else None, gy if need[1] else None, dw1, db1, dw2,
                db2, None, None, None)


def fused_ff_supported(x, w1, w2):
    return (FUSED_FF and x.is_cuda and x.shape[-1] == 128 and tuple(w1.shape) == (128, 128)
            and tuple(w2.shape) == (128, 128))


def fused_ff(xn, r, w1, b1, w2, b2, gate, p, site):
    return _FusedFF.apply(xn, r, w1, b1, w2, b2, gate, float(p), int(site))


# ---------------------------------------------------------------- fused attention branch
FUSED_ATTN = True


class _AttnBranch(torch.autograd.Function):
    """x + gate * Attention(RMSNorm(x)) for the LF prior's width (128, 2 heads of 64, S <= 32)
    in one launch forward and one backward (csrc/tvq_xattn.hip; x-transformers pre-norm
    attention layer, bidirectional_transformer.py:92-110).  The weight gradients go through
    the grouped weight-gradient path like every Linear's: dWqkv = dqkv^T xn into the stacked
    flat-gradient view (as _QKVAttention), dWo = (gate gy)^T o; the RMSNorm gain gradient is a
    deferred slab sum."""

    @staticmethod
    def forward(ctx, x, g, wq, wk, wv, wo, gate, heads, p, site):
        B, S, D = x.shape
        M = B * S
        x2 = x.reshape(M, D).contiguous()
        W = _stacked([wq, wk, wv], (3 * D, D))
        if W is None:
            W = torch.cat([wq, wk, wv], 0).contiguous()
        dev = x.device
        y, xn, o = (torch.empty_like(x2) for _ in range(3))
        inv = torch.empty(M, device=dev)
        qkv = torch.empty((M, 3 * D), device=dev)
        lse = torch.empty(B * heads * S, device=dev)
        seed = rng.seed_tensor(dev) if p > 0 else None
        off = rng.call_offset(site) if p > 0 else 0
        call("tvq_attn_branch_fwd", ptr(x2), B, S, D, heads, ptr(g), math.sqrt(D), ptr(W), ptr(wo),
             ptr(gate), float(p), ptr(seed), off, ptr(y), ptr(xn), ptr(inv), ptr(qkv), ptr(o),
             ptr(lse), stream_ptr())
        ctx.save_for_backward(x2, xn, inv, qkv, o, lse, W)
        ctx.params = (wq, wk, wv, wo, g)
        ctx.gate, ctx.seed = gate, seed
        ctx.cfg = (B, S, D, heads, float(p), off)
        ctx.wg_tag = wgrad.current_tag()
        return y.reshape(B, S, D)

    @staticmethod
    def backward(ctx, gy):
        x2, xn, inv, qkv, o, lse, W = ctx.saved_tensors
        B, S, D, heads, p, off = ctx.cfg
        wq, wk, wv, wo, g = ctx.params
        M, L = B * S, 3 * D
        dev = x2.device
        g2 = gy.reshape(M, D).contiguous()
        need = ctx.needs_input_grad
        dx = torch.empty_like(x2)
        dqkv = torch.empty((M, L), device=dev)
        gg = torch.empty_like(g2) if ctx.gate is not None else None
        sink_g = grad_sink(g)
        dg = sink_g if sink_g is not None else torch.empty(D, device=dev)
        ws = torch.empty(value("tvq_attn_branch_workspace", B, D), device=dev)
        call("tvq_attn_branch_bwd", ptr(g2), ptr(x2), B, S, D, heads, ptr(g), math.sqrt(D), ptr(inv),
             ptr(W), ptr(wo), ptr(ctx.gate), p, ptr(ctx.seed), off, ptr(qkv), ptr(o), ptr(lse),
             ptr(dx), ptr(dqkv), ptr(gg), ptr(dg), int(sink_g is not None), ptr(ws), stream_ptr())
        _keep(ws)  # its gain-gradient reduction may be deferred
        dws = [None, None, None]
        if any(need[2:5]):
            sinks = [grad_sink(w) for w in (wq, wk, wv)]
            sink = _stacked(sinks, (L, D)) if all(s_ is not None for s_ in sinks) else None
            if sink is not None:  # into the flat gradient (stacked view)
                if not wgrad.defer(dqkv, L, xn, D, sink, D, L, D, M, ctx.wg_tag):
                    with streams.offload(dqkv, xn):
                        gemm(dqkv, 1, L, xn, D, 1, L, D, M, out=sink, ldc=D, accumulate=True)
            else:
                dW = gemm(dqkv, 1, L, xn, D, 1, L, D, M)
                dws = [dW[i * D:(i + 1) * D] for i in range(3)]
        dwo = weight_grad(gg if gg is not None else g2, o, wo, M, D, D, ctx.wg_tag) if need[5] else None
        return (dx.reshape(B, S, D), None if sink_g is not None else dg, *dws, dwo, None, None, None,
                None)


def attn_branch_supported(x, g, attn):
    """Whether the fused attention branch (tvq_attn_branch_*) takes this layer: width 128,
    2 heads of 64, <= 32 tokens, fp32 device weights on 16-byte boundaries."""
    if not (FUSED_ATTN and x.is_cuda and x.dim() == 3 and x.shape[-1] == 128 and x.shape[1] <= 32
            and attn.heads == 2):
        return False
    ws = (g, attn.to_q.weight, attn.to_k.weight, attn.to_v.weight, attn.to_out.weight)
    return all(w.dtype == torch.float32 and w.is_cuda and w.is_contiguous() and
               w.data_ptr() % 16 == 0 for w in ws) and tuple(attn.to_q.weight.shape) == (128, 128)


def attn_branch(x, g, attn, gate, p):
    """x + gate * attn(RMSNorm_g(x)) (pre-norm residual attention layer) on the fused path."""
    return _AttnBranch.apply(x, g, attn.to_q.weight, attn.to_k.weight, attn.to_v.weight,
                             attn.to_out.weight, gate, int(attn.heads), float(p), int(attn._site))


# ---------------------------------------------------------------- attention
class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, heads, drop_p, site):
        # q/k/v: (B, S, heads*64) contiguous
        B, S, HD = q.shape
        Dh = HD // heads
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        o = torch.empty_like(q)
        lse = torch.empty(B * heads * S, device=q.device)
        seed = rng.seed_tensor(q.device) if drop_p > 0 else None
        off = rng.call_offset(site) if drop_p > 0 else 0
        scale = Dh ** -0.5
        call("tvq_attention_fwd", ptr(q), HD, ptr(k), HD, ptr(v), HD, ptr(o), HD, ptr(lse), B,
             heads, S, Dh, float(scale), float(drop_p), ptr(seed), off, stream_ptr())
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.cfg = (heads, drop_p, off, scale)
        ctx.seed = seed
        return o

    @staticmethod
    def backward(ctx, go):
        q, k, v, o, lse = ctx.saved_tensors
        heads, drop_p, off, scale = ctx.cfg
        B, S, HD = q.shape
        Dh = HD // heads
        go = go.contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        call("tvq_attention_bwd", ptr(q), HD, ptr(k), HD, ptr(v), HD, ptr(o), HD, ptr(go), HD,
             ptr(lse), B,
             heads, S, Dh, float(scale), float(drop_p), ptr(ctx.seed), off, ptr(dq), ptr(dk),
             ptr(dv), HD, stream_ptr())
        return dq, dk, dv, None, None, None


def attention(q, k, v, heads, drop_p=0.0, site=0):
    """softmax(q k^T / sqrt(64)) [dropout] v per head; q/k/v (B, S, heads*64)."""
    return _Attention.apply(q, k, v, int(heads), float(drop_p), int(site))


def _stacked(ws, shape):
    """The row-stacked matrix of `ws` as one view when they are consecutive in memory
    (FusedAdamW's flat buffers keep to_q, to_k, to_v adjacent), else None."""
    p0 = ws[0]
    if any(w is None or not w.is_contiguous() for w in ws):
        return None
    step = p0.numel() * p0.element_size()
    base = p0.untyped_storage().data_ptr()
    if any(w.untyped_storage().data_ptr() != base or w.data_ptr() != p0.data_ptr() + i * step
           for i, w in enumerate(ws)):
        return None  # separate storages (adjacent allocations are not one buffer)
    return torch.as_strided(p0, shape, (shape[1], 1))


class _QKVAttention(torch.autograd.Function):
    """o = attention(x Wq^T, x Wk^T, x Wv^T): the three projections as ONE GEMM against the
    row-stacked [Wq; Wk; Wv] (a view of the flat parameters when they are adjacent), the
    attention reading q / k / v as strided column blocks of its output; the backward
    writes dq | dk | dv into one buffer, then one input-gradient GEMM and one weight-
    gradient GEMM (straight into the stacked flat-gradient view) replace three of each
    and their two accumulation adds."""

    @staticmethod
    def forward(ctx, x, wq, wk, wv, heads, drop_p, site):
        B, S, D = x.shape
        HD = wq.shape[0]
        x2 = x.reshape(B * S, D).contiguous()
        M = B * S
        W = _stacked([wq, wk, wv], (3 * HD, D))
        if W is None:
            W = torch.cat([wq, wk, wv], 0).contiguous()
        qkv = gemm(x2, D, 1, W, 1, D, M, 3 * HD, D)
        Dh = HD // heads
        o = torch.empty((M, HD), device=x.device)
        lse = torch.empty(B * heads * S, device=x.device)
        seed = rng.seed_tensor(x.device) if drop_p > 0 else None
        off = rng.call_offset(site) if drop_p > 0 else 0
        scale = Dh ** -0.5
        L = 3 * HD
        call("tvq_attention_fwd", ptr(qkv), L, ptr(qkv[:, HD:]), L, ptr(qkv[:, 2 * HD:]), L, ptr(o),
             HD, ptr(lse), B, heads, S, Dh, float(scale), float(drop_p), ptr(seed), off,
             stream_ptr())
        ctx.save_for_backward(x2, W, qkv, o, lse)
        ctx.params = (wq, wk, wv)
        ctx.wg_tag = wgrad.current_tag()
        ctx.cfg = (B, S, D, HD, heads, drop_p, off, scale)
        ctx.seed = seed
        return o.reshape(B, S, HD)

    @staticmethod
    def backward(ctx, go):
        x2, W, qkv, o, lse = ctx.saved_tensors
        B, S, D, HD, heads, drop_p, off, scale = ctx.cfg
        M, L, Dh = B * S, 3 * HD, HD // heads
        go = go.reshape(M, HD).contiguous()
        dqkv = torch.empty((M, L), device=go.device)
        call("tvq_attention_bwd", ptr(qkv), L, ptr(qkv[:, HD:]), L, ptr(qkv[:, 2 * HD:]), L, ptr(o),
             HD, ptr(go), HD, ptr(lse), B, heads, S, Dh, float(scale), float(drop_p),
             ptr(ctx.seed), off, ptr(dqkv), ptr(dqkv[:, HD:]), ptr(dqkv[:, 2 * HD:]), L,
             stream_ptr())
        dx = None
        if ctx.needs_input_grad[0]:
            dx = gemm(dqkv, L, 1, W, D, 1, M, D, L).reshape(B, S, D)
        dws = [None, None, None]
        if any(ctx.needs_input_grad[1:4]):
            sinks = [grad_sink(p) for p in ctx.params]
            sink = _stacked(sinks, (L, D)) if all(s is not None for s in sinks) else None
            if sink is not None:  # into the flat gradient (stacked view)
                if not wgrad.defer(dqkv, L, x2, D, sink, D, L, D, M, ctx.wg_tag):  # else grouped later
                    with streams.offload(dqkv, x2):
                        gemm(dqkv, 1, L, x2, D, 1, L, D, M, out=sink, ldc=D, accumulate=True)
            else:
                dW = gemm(dqkv, 1, L, x2, D, 1, L, D, M)
                dws = [dW[i * HD:(i + 1) * HD] for i in range(3)]
        return (dx, *dws, None, None, None)


def qkv_attention(x, wq, wk, wv, heads, drop_p=0.0, site=0):
    """attention(x Wq^T, x Wk^T, x Wv^T) with the projections fused (_QKVAttention)."""
    return _QKVAttention.apply(x, wq, wk, wv, int(heads), float(drop_p), int(site))


# ---------------------------------------------------------------- embedding
class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, table, mask_id, drop_p, site):
        idx = idx.contiguous()
        M = idx.numel()
        V, D = table.shape
        out = torch.empty((M, D), device=table.device)
        seed = rng.seed_tensor(table.device) if drop_p > 0 else None
        off = rng.call_offset(site) if drop_p > 0 else 0
        call("tvq_embedding_fwd", ptr(idx), M, D, ptr(table), ptr(out), D, int(mask_id),
             float(drop_p), ptr(seed), off, stream_ptr())
        ctx.save_for_backward(idx)
        ctx.table = table
        ctx.cfg = (V, D, mask_id, drop_p, off)
        ctx.seed = seed
        return out.reshape(*idx.shape, D)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        V, D, mask_id, drop_p, off = ctx.cfg
        M = idx.numel()
        g2 = g.reshape(M, D).contiguous()
        sink = grad_sink(ctx.table)
        # into the flat gradient: aux stream (same one as the tied-logits table grad)
        with (streams.offload(idx, g2) if sink is not None else contextlib.nullcontext()):
            tg = sink if sink is not None else torch.empty((V, D), device=g.device)
            ws = torch.empty(value("tvq_embedding_bwd_workspace", M, V), device=g.device,
                             dtype=torch.int32)
            call("tvq_embedding_bwd", ptr(idx), M, D, ptr(g2), D, V, ptr(tg),
                 int(sink is not None), int(mask_id), float(drop_p), ptr(ctx.seed), off, ptr(ws),
                 stream_ptr())
        return None, (None if sink is not None else tg), None, None, None


def embedding(idx, table, mask_id=-1, drop_p=0.0, site=0):
    """table[idx] with dropout on positions where idx != mask_id (mask_id=-1: everywhere)."""
    return _Embedding.apply(idx, table, int(mask_id), float(drop_p), int(site))


# ------------------------------------------------------- embedding assembly
class _EmbedAssemble(torch.autograd.Function):
    """cat(cls_emb, [t1 | t2] + pos[:n], dim=1) in one kernel (bidirectional_transformer.py:
    185,229-231); the backward splits the gradient back into the inputs' own layouts (the
    Upscale output is a transposed view) and sums the position-table gradient over the
    batch in order into its flat-gradient rows."""

    @staticmethod
    def forward(ctx, cls_emb, t1, t2, pos_w, n):
        B, _, D1 = t1.shape
        D2 = t2.shape[-1] if t2 is not None else 0
        Dt = D1 + D2
        cls2 = cls_emb.reshape(B, Dt).contiguous()
        out = torch.empty((B, n + 1, Dt), device=t1.device)
        s2 = t2.stride() if t2 is not None else (0, 0, 0)
        call("tvq_embed_assemble", ptr(cls2), ptr(t1), *t1.stride(), D1, ptr(t2), *s2, D2,
             ptr(pos_w), B, n, ptr(out), stream_ptr())
        ctx.meta = (B, n, D1, D2, tuple(t1.shape), t1.stride(),
                    None if t2 is None else (tuple(t2.shape), t2.stride()), tuple(cls_emb.shape))
        ctx.pos_w = pos_w
        return out

    @staticmethod
    def backward(ctx, g):
        B, n, D1, D2, sh1, st1, m2, shc = ctx.meta
        g = g.contiguous()
        dev = g.device
        need = ctx.needs_input_grad
        dcls = torch.empty(shc, device=dev) if need[0] else None
        dt1 = torch.empty_strided(sh1, st1, device=dev) if need[1] else None
        dt2 = torch.empty_strided(m2[0], m2[1], device=dev) if (m2 is not None and need[2]) else None
        s2 = m2[1] if m2 is not None else (0, 0, 0)
        sink = grad_sink(ctx.pos_w) if need[3] else None
        dpos = None
        if need[3]:
            dpos = sink if sink is not None else torch.zeros_like(ctx.pos_w)
        call("tvq_embed_assemble_bwd", ptr(g), B, n, D1, D2, ptr(dcls), ptr(dt1), *st1, ptr(dt2),
             *s2, ptr(dpos), int(sink is not None), stream_ptr())
        return dcls, dt1, dt2, (None if sink is not None else dpos), None


def embed_assemble(cls_emb, t1, t2, pos_w, n):
    """cat(cls_emb (B,1,D), [t1 | t2] + pos_w[:n], dim=1) -> (B, n+1, D) (t2 may be None)."""
    return _EmbedAssemble.apply(cls_emb, t1, t2, pos_w, int(n))


# ---------------------------------------------------------------- masked CE
class _MaskedCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, keep):
        K = logits.shape[-1]
        l2 = logits.reshape(-1, K).contiguous()
        M = l2.shape[0]
        t = target.reshape(-1).contiguous()
        kp = keep.reshape(-1).contiguous()
        lse = torch.empty(M, device=logits.device)
        out = torch.empty(2, device=logits.device)
        ws = torch.empty(value("tvq_masked_ce_workspace", M), device=logits.device)
        call("tvq_masked_ce_fwd", ptr(l2), K, M, K, ptr(t), ptr(kp), ptr(lse), ptr(out), ptr(ws),
             stream_ptr())
        ctx.save_for_backward(l2, t, kp, lse, out)
        ctx.shape = logits.shape
        return out[0]

    @staticmethod
    def backward(ctx, g):
        l2, t, kp, lse, stats = ctx.saved_tensors
        M, K = l2.shape
        dl = torch.empty_like(l2)
        g = g.reshape(1).contiguous()
        call("tvq_masked_ce_bwd", ptr(l2), K, M, K, ptr(t), ptr(kp), ptr(lse), ptr(stats), ptr(g),
             ptr(dl), K, stream_ptr())
        return dl.reshape(ctx.shape), None, None


def masked_cross_entropy(logits, target, keep):
    """F.cross_entropy(logits[~keep], target[~keep]) (maskgit.py:183-191)."""
    return _MaskedCE.apply(logits, target, keep)


def mask_tokens(s, mask_id, site, ratio=None, rand=None):
    """_randomly_mask_tokens on device; returns (s_M int64, keep bool)."""
    s = s.contiguous()
    B, n = s.shape
    s_M = torch.empty_like(s)
    keep = torch.empty((B, n), device=s.device, dtype=torch.bool)
    seed = rng.seed_tensor(s.device)
    call("tvq_mask_tokens", ptr(s), B, n, int(mask_id), ptr(seed), rng.call_offset(site),
         ptr(ratio.to(torch.float64).contiguous() if ratio is not None else None),
         ptr(rand.contiguous() if rand is not None else None), ptr(s_M), ptr(keep), stream_ptr())
    return s_M, keep


# ---------------------------------------------------------------- misc
class _UpNearest(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, Lout):
        x = x.contiguous()
        Lin = x.shape[-1]
        R = x.numel() // Lin
        y = torch.empty((*x.shape[:-1], Lout), device=x.device)
        call("tvq_upsample_nearest", ptr(x), R, Lin, Lout, ptr(y), stream_ptr())
        ctx.cfg = (x.shape, R, Lin, Lout)
        return y

    @staticmethod
    def backward(ctx, gy):
        shape, R, Lin, Lout = ctx.cfg
        g = gy.contiguous()
        dx = torch.empty(shape, device=g.device)
        call("tvq_upsample_nearest_bwd", ptr(g), R, Lin, Lout, ptr(dx), stream_ptr())
        return dx, None


def upsample_nearest(x, size):
    return _UpNearest.apply(x, int(size))


class _UpNearestT(torch.autograd.Function):
    """(b, n, d) -> transpose -> nearest upsample to m -> (b, d, m), one pass each way."""

    @staticmethod
    def forward(ctx, x, Lout):
        x = x.contiguous()
        B, Lin, D = x.shape
        y = torch.empty((B, D, Lout), device=x.device)
        call("tvq_upsample_nearest_t", ptr(x), B, Lin, D, Lout, ptr(y), stream_ptr())
        ctx.cfg = (B, Lin, D, Lout)
        return y

    @staticmethod
    def backward(ctx, gy):
        B, Lin, D, Lout = ctx.cfg
        g = gy.contiguous()
        dx = torch.empty((B, Lin, D), device=g.device)
        call("tvq_upsample_nearest_t_bwd", ptr(g), B, Lin, D, Lout, ptr(dx), stream_ptr())
        return dx, None


def upsample_nearest_t(x, size):
    """F.interpolate(x.transpose(1, 2), size, mode='nearest') for x (b, n, d) -> (b, d, size)."""
    return _UpNearestT.apply(x, int(size))


def batch_colsum(x, out, ldo, accumulate):
    """out[j*ldo + d] (+)= sum_b x[b, j, d] for x (B, n, D) contiguous (tvq_batch_colsum)."""
    B, n, D = x.shape
    call("tvq_batch_colsum", ptr(x), B, n * D, n, D, D, ptr(out), ldo, int(bool(accumulate)),
         stream_ptr())


class _GELU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        call("tvq_gelu_fwd", ptr(x), x.numel(), ptr(y), stream_ptr())
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        g = gy.contiguous()
        dx = torch.empty_like(x)
        call("tvq_gelu_bwd", ptr(g), ptr(x), x.numel(), ptr(dx), stream_ptr())
        return dx


def gelu(x):
    return _GELU.apply(x)


# --------------------------------------------------------------------------- fused LF prior
PRIOR_FUSED = True


def prior_lf_eval_supported(tf, s):
    """Whether BidirectionalTransformer `tf` (an LF prior in eval mode, no gradient needed)
    matches tvq_prior_lf_eval: width 128 everywhere (embed = hidden = heads * 64 = ff inner),
    RMSNorm layers, depth <= 8, n + 1 <= 32 tokens, fp32 device weights."""
    if not PRIOR_FUSED or tf.kind != "lf" or tf.training or not s.is_cuda:
        return False
    if torch.is_grad_enabled() and any(p.requires_grad for p in tf.parameters()):
        return False
    enc = tf.blocks.attn_layers
    if enc.dim != 128 or tf.tok_emb_l.weight.shape[1] != 128 or len(enc.layers) > 16:
        return False
    if s.dim() != 2 or s.shape[1] + 1 > 32 or s.shape[1] != tf.num_tokens:
        return False
    for i, (norms, block, _) in enumerate(enc.layers):
        if not hasattr(norms[0], "scale"):  # RMSNorm
            return False
        if i % 2 == 0:  # ("a", "f") * depth
            if not hasattr(block, "to_q") or block.heads * 64 != 128:
                return False
        elif not hasattr(block, "ff") or block.ff[0][0].weight.shape[0] != 128:
            return False
    # tvq_prior_lf_eval reads every weight with 16-byte loads (TVQ_CHECK_ARG there): a
    # FusedAdamW flat buffer packs parameters without padding, so check, don't assume
    return all(p.dtype == torch.float32 and p.is_cuda and p.is_contiguous() and
               p.data_ptr() % 16 == 0 for p in tf.parameters())


def _prior_lf_args(tf, s, class_idx, ws=None):
    import ctypes
    enc = tf.blocks.attn_layers
    w = [tf.tok_emb_l.weight, tf.pos_emb.weight, tf.class_condition_emb.weight,
         tf.blocks.project_in.weight, tf.blocks.post_emb_norm.gamma]
    for i in range(0, len(enc.layers), 2):
        na, attn, _ = enc.layers[i]
        nf, ff, _ = enc.layers[i + 1]
        w += [na[0].g, attn.to_q.weight, attn.to_k.weight, attn.to_v.weight, attn.to_out.weight,
              nf[0].g, ff.ff[0][0].weight, ff.ff[0][0].bias, ff.ff[2].weight, ff.ff[2].bias]
    w += [enc.final_norm.g, tf.blocks.project_out.weight, tf.pred_head[0].weight,
          tf.pred_head[0].bias, tf.pred_head[2].weight, tf.pred_head[2].bias, tf.bias]
    arr = (ctypes.c_void_p * len(w))(*[ptr(t) for t in w])
    s = s if s.stride(1) == 1 else s.contiguous()
    cls = class_idx.reshape(-1).long().contiguous() if class_idx is not None else None
    depth = len(enc.layers) // 2
    K = tf.codebook_size
    if ws is None:
        ws = prior_lf_eval_workspace(tf, s)
    return s, cls, arr, depth, K, ws


def prior_lf_eval_workspace(tf, s):
    """The packed-weight workspace of tvq_prior_lf_eval(_sample) for prior `tf` and tokens
    like `s` (reusable across calls with the same weights: see prior_lf_eval_sample)."""
    depth = len(tf.blocks.attn_layers.layers) // 2
    return torch.empty(value("tvq_prior_lf_eval_workspace", depth, tf.codebook_size, s.shape[1],
                             tf.n_classes), device=s.device, dtype=torch.uint8)


def prior_lf_eval(tf, s, class_idx=None):
    """logits (B, n, K) of the LF prior in eval mode as ONE launch (csrc/tvq_prior_eval.hip):
    the same function as forward_lf's unfused path (embedding, encoder, pred_head, tied
    logits).  class_idx: (B,) / (B, 1) int64 or None (the null class)."""
    s, cls, arr, depth, K, ws = _prior_lf_args(tf, s, class_idx)
    B, n = s.shape
    logits = torch.empty((B, n, K), device=s.device, dtype=torch.float32)
    call("tvq_prior_lf_eval", ptr(s), B, n, s.stride(0), ptr(cls), tf.n_classes, 128, arr,
         depth, K, float(tf.pred_head[2].eps), ptr(logits), ptr(ws), stream_ptr())
    return logits


def prior_lf_eval_sample(tf, s, class_idx, mask_id, gumbel=None, site=0, want_logits=False,
                         ws=None, ready=False):
    """prior_lf_eval + hip.sample.maskgit_sample in ONE launch: the tied logits are drawn
    from by the race in registers and never written (tvq_prior_lf_eval_sample).  Returns
    (sampled, p(sampled)[, logits]).  ws / ready: a workspace from an earlier call with the
    same weights (ready=True skips packing them again: the decoding steps after the first)."""
    from . import rng
    s, cls, arr, depth, K, ws = _prior_lf_args(tf, s, class_idx, ws)
    B, n = s.shape
    dev = s.device
    sampled = torch.empty((B, n), device=dev, dtype=torch.int64)
    selp = torch.empty((B, n), device=dev, dtype=torch.float32)
    logits = torch.empty((B, n, K), device=dev, dtype=torch.float32) if want_logits else None
    seed = rng.seed_tensor(dev) if gumbel is None else None
    off = rng.call_offset(site) if gumbel is None else 0
    call("tvq_prior_lf_eval_sample", ptr(s), B, n, s.stride(0), ptr(cls), tf.n_classes, 128, arr,
         depth, K, float(tf.pred_head[2].eps), int(mask_id),
         ptr(gumbel.contiguous() if gumbel is not None else None), ptr(seed), off,
         ptr(sampled), ptr(selp), ptr(logits), ptr(ws), int(bool(ready)), stream_ptr())
    return (sampled, selp, logits) if want_logits else (sampled, selp)


class _DropFirst(torch.autograd.Function):
    """x[:, 1:, :] as a contiguous tensor (tvq_drop_first_token), its backward one kernel
    writing the zero class rows (instead of a PyTorch copy, fill and copy)."""

    @staticmethod
    def forward(ctx, x):
        B, n1, D = x.shape
        x = x.contiguous()
        y = torch.empty((B, n1 - 1, D), device=x.device, dtype=x.dtype)
        call("tvq_drop_first_token", ptr(x), B, n1 - 1, D, ptr(y), 0, stream_ptr())
        return y

    @staticmethod
    def backward(ctx, g):
        B, n, D = g.shape
        g = g.contiguous()
        dx = torch.empty((B, n + 1, D), device=g.device, dtype=g.dtype)
        call("tvq_drop_first_token", ptr(g), B, n, D, ptr(dx), 1, stream_ptr())
        return dx


def drop_first_token(x):
    """embed[:, 1:, :] (B, n+1, D) -> (B, n, D) contiguous on the HIP path."""
    if x.shape[-1] % 4 or not x.is_cuda:
        return x[:, 1:, :].contiguous()
    return _DropFirst.apply(x)
