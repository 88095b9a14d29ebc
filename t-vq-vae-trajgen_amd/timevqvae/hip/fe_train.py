"""FidelityEnhancer training ops (Stage3, trainers/stage3.py:197-231) on the HIP path.

Autograd functions over csrc/tvq_fe_train.hip (backward kernels, the GroupNorm+Snake
training forward with the Block's dropout) and the eval kernels of csrc/tvq_fe.hip whose
forward is unchanged in training (channel LayerNorm, both attention cores,
interpolate+concat).  The Unet1D convolutions train on the conv engine (hip.conv.conv2d
with H = 1: fused bias / residual epilogues, deterministic weight gradients).
Every per-channel parameter gradient is a fixed-order channel sum (tvq_channel_sum).
"""
import torch

from . import rng
from ._native import call, ptr, stream_ptr, value


def _c(t):
    return t.contiguous()


def _chan_sum(t, out=None):
    """sum over (b, l) per channel of a (B, C, L) tensor."""
    B, C, L = t.shape
    o = out if out is not None else torch.empty(C, device=t.device, dtype=torch.float32)
    ws = torch.empty(max(1, value("tvq_channel_sum_workspace", B, C, L)), device=t.device)
    call("tvq_channel_sum", ptr(t), B, C, L, ptr(o), 0, ptr(ws), stream_ptr())
    return o


# ---------------------------------------------------------------- weight standardisation
class _WS(torch.autograd.Function):
    @staticmethod
    def forward(ctx, w, eps):
        w = _c(w)
        out = torch.empty_like(w)
        call("tvq_fe_ws_weight", ptr(w), w.shape[0], w[0].numel(), float(eps), ptr(out),
             stream_ptr())
        ctx.save_for_backward(w)
        ctx.eps = eps
        return out

    @staticmethod
    def backward(ctx, g):
        (w,) = ctx.saved_tensors
        dw = torch.empty_like(w)
        call("tvq_fe_ws_weight_bwd", ptr(w), w.shape[0], w[0].numel(), float(ctx.eps), ptr(_c(g)),
             ptr(dw), 0, stream_ptr())
        return dw, None


def standardize_weight(w, eps=1e-5):
    """WeightStandardizedConv2d's weight (fidelity_enhancer.py:102-106), differentiable."""
    return _WS.apply(w, float(eps))


# ---------------------------------------------------------------- GroupNorm + Snake (+drop)
class _GNSnake(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, a, residual, groups, eps, drop_p, site):
        x = _c(x)
        B, C, L = x.shape
        y = torch.empty_like(x)
        mean = torch.empty(B * groups, device=x.device)
        rstd = torch.empty(B * groups, device=x.device)
        seed = rng.seed_tensor(x.device) if drop_p > 0 else None
        off = rng.call_offset(site) if drop_p > 0 else 0
        res = _c(residual) if residual is not None else None
        call("tvq_fe_gn_snake_train_fwd", ptr(x), B, C, L, int(groups), ptr(_c(gamma)),
             ptr(_c(beta)), ptr(_c(a).reshape(-1)), float(eps), float(drop_p), ptr(seed), off,
             ptr(res), ptr(y), ptr(mean), ptr(rstd), stream_ptr())
        ctx.save_for_backward(x, gamma, beta, a, mean, rstd)
        ctx.cfg = (int(groups), float(drop_p), off, residual is not None)
        ctx.seed = seed
        return y

    @staticmethod
    def backward(ctx, gy):
        x, gamma, beta, a, mean, rstd = ctx.saved_tensors
        groups, drop_p, off, has_res = ctx.cfg
        B, C, L = x.shape
        g = _c(gy)
        dx, tg, tb, ta = (torch.empty_like(x) for _ in range(4))
        call("tvq_fe_gn_snake_bwd", ptr(g), ptr(x), B, C, L, groups, ptr(_c(gamma)), ptr(_c(beta)),
             ptr(_c(a).reshape(-1)), ptr(mean), ptr(rstd), float(drop_p), ptr(ctx.seed), off,
             ptr(dx), ptr(tg), ptr(tb), ptr(ta), stream_ptr())
        dgam, dbet = _chan_sum(tg), _chan_sum(tb)
        da = _chan_sum(ta).view_as(a)
        return dx, dgam, dbet, da, (gy if has_res else None), None, None, None, None


def group_norm_snake(x, groups, gamma, beta, a, eps=1e-5, residual=None, drop_p=0.0, site=0):
    """Dropout_p(Snake(GroupNorm(x))) (+ residual): Block.forward in training
    (fidelity_enhancer.py:193-204) with the ResnetBlock skip add (:231)."""
    return _GNSnake.apply(x, gamma, beta, a, residual, int(groups), float(eps), float(drop_p),
                          int(site))


# ---------------------------------------------------------------- channel LayerNorm
class _ChanLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, residual, eps):
        x = _c(x)
        B, C, L = x.shape
        y = torch.empty_like(x)
        res = _c(residual) if residual is not None else None
        call("tvq_fe_channel_layernorm", ptr(x), B, C, L, ptr(_c(g).reshape(-1)), float(eps),
             ptr(res), ptr(y), stream_ptr())
        ctx.save_for_backward(x, g)
        ctx.eps, ctx.has_res = eps, residual is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, g = ctx.saved_tensors
        B, C, L = x.shape
        dx, tg = torch.empty_like(x), torch.empty_like(x)
        call("tvq_fe_channel_layernorm_bwd", ptr(_c(gy)), ptr(x), B, C, L, ptr(_c(g).reshape(-1)),
             float(ctx.eps), ptr(dx), ptr(tg), stream_ptr())
        return dx, _chan_sum(tg).view_as(g), (gy if ctx.has_res else None), None


def channel_layernorm(x, g, eps=1e-5, residual=None):
    """LayerNorm over channels with gain g (:119-127) (+ residual), differentiable."""
    return _ChanLN.apply(x, g, residual, float(eps))


# ---------------------------------------------------------------- attention cores
class _AttnCore(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads, dim_head, linear):
        qkv = _c(qkv)
        B, C3, n = qkv.shape
        out = torch.empty((B, heads * dim_head, n), device=qkv.device, dtype=torch.float32)
        call("tvq_fe_linear_attention" if linear else "tvq_fe_attention", ptr(qkv), B, heads,
             dim_head, n, ptr(out), stream_ptr())
        ctx.save_for_backward(qkv)
        ctx.cfg = (heads, dim_head, linear)
        return out

    @staticmethod
    def backward(ctx, gout):
        (qkv,) = ctx.saved_tensors
        heads, dim_head, linear = ctx.cfg
        B, C3, n = qkv.shape
        dqkv = torch.empty_like(qkv)
        call("tvq_fe_linear_attention_bwd" if linear else "tvq_fe_attention_bwd", ptr(qkv),
             ptr(_c(gout)), B, heads, dim_head, n, ptr(dqkv), stream_ptr())
        return dqkv, None, None, None


def linear_attention(qkv, heads, dim_head):
    """LinearAttention core (:245-258), differentiable."""
    return _AttnCore.apply(qkv, int(heads), int(dim_head), True)


def attention(qkv, heads, dim_head):
    """Attention core (:273-282), differentiable."""
    return _AttnCore.apply(qkv, int(heads), int(dim_head), False)


# ---------------------------------------------------------------- interpolate + concat
class _CatInterp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, length):
        a = _c(a)
        B, Ca, La = a.shape
        if b is not None:
            b = _c(b)
            Cb, Lb = b.shape[1], b.shape[2]
        else:
            Cb, Lb = 0, 0
        out = torch.empty((B, Ca + Cb, int(length)), device=a.device, dtype=torch.float32)
        call("tvq_fe_cat_interp", ptr(a), Ca, La, ptr(b), Cb, Lb, B, int(length), ptr(out),
             stream_ptr())
        ctx.cfg = (B, Ca, La, Cb, Lb, int(length))
        return out

    @staticmethod
    def backward(ctx, g):
        B, Ca, La, Cb, Lb, L = ctx.cfg
        da = torch.empty((B, Ca, La), device=g.device)
        db = torch.empty((B, Cb, Lb), device=g.device) if Cb else None
        call("tvq_fe_cat_interp_bwd", ptr(_c(g)), Ca, La, Cb, Lb, B, L, ptr(da), ptr(db),
             stream_ptr())
        return da, db, None


def cat_interp(a, b, length):
    """cat(interp(a, length), interp(b, length)) (:434-452, 495-497), differentiable."""
    return _CatInterp.apply(a, b, int(length))
