"""FidelityEnhancer / Unet1D ops on the HIP path (csrc/tvq_fe.hip, include/tvq.h).

Eval-mode forward only: the reference runs the FidelityEnhancer under no_grad in the
sampler (generation/sampler.py:156-169).  Every op allocates its output with torch
(the caching allocator) and launches on the current stream; none falls back to torch
arithmetic."""
import torch

from ._native import call, ptr, stream_ptr, value


def _c(t):
    return t.detach().contiguous()


def conv1d(x, weight, bias=None, stride=1, padding=0, upsample2=False, replicate=False,
           residual=None, standardize=False, eps=1e-5):
    """nn.Conv1d (fidelity_enhancer.py:85-116,386-392): optional weight standardisation
    (WeightStandardizedConv2d), nearest-x2 input, replicate padding, fused residual."""
    x, w = _c(x), _c(weight)
    B, Ci, Lin = x.shape
    Co, Ci_w, K = w.shape
    if Ci_w != Ci:
        raise ValueError(f"conv1d: weight expects {Ci_w} input channels, got {Ci}")
    s = stream_ptr()
    if standardize:
        ws = torch.empty_like(w)
        call("tvq_fe_ws_weight", ptr(w), Co, Ci * K, float(eps), ptr(ws), s)
        w = ws
    Lout = value("tvq_fe_conv1d_out_len", Lin, K, stride, padding, int(upsample2))
    y = torch.empty((B, Co, Lout), device=x.device, dtype=torch.float32)
    res = _c(residual) if residual is not None else None
    if res is not None and res.shape != y.shape:
        raise ValueError(f"conv1d: residual {tuple(res.shape)} != output {tuple(y.shape)}")
    call("tvq_fe_conv1d", ptr(x), B, Ci, Lin, ptr(w), ptr(_c(bias) if bias is not None else None),
         Co, K, int(stride), int(padding), int(upsample2), int(replicate), ptr(res), ptr(y), Lout, s)
    return y


def standardize_weight(weight, eps=1e-5):
    """WeightStandardizedConv2d's weight (fidelity_enhancer.py:102-106) on the device."""
    w = _c(weight)
    out = torch.empty_like(w)
    call("tvq_fe_ws_weight", ptr(w), w.shape[0], w[0].numel(), float(eps), ptr(out), stream_ptr())
    return out


def group_norm_snake(x, groups, gamma, beta, a, eps=1e-5, residual=None):
    """GroupNorm -> Snake (+ residual): Block.forward + ResnetBlock skip (:193-231)."""
    x = _c(x)
    B, C, L = x.shape
    y = torch.empty_like(x)
    res = _c(residual) if residual is not None else None
    call("tvq_fe_group_norm_snake", ptr(x), B, C, L, int(groups), ptr(_c(gamma)), ptr(_c(beta)),
         ptr(_c(a).reshape(-1)), float(eps), ptr(res), ptr(y), stream_ptr())
    return y


def channel_layernorm(x, g, eps=1e-5, residual=None):
    """LayerNorm over channels, gamma only (:119-127) (+ residual)."""
    x = _c(x)
    B, C, L = x.shape
    y = torch.empty_like(x)
    res = _c(residual) if residual is not None else None
    call("tvq_fe_channel_layernorm", ptr(x), B, C, L, ptr(_c(g).reshape(-1)), float(eps), ptr(res),
         ptr(y), stream_ptr())
    return y


def _attn(name, qkv, heads, dim_head):
    qkv = _c(qkv)
    B, C3, n = qkv.shape
    if C3 != 3 * heads * dim_head:
        raise ValueError(f"{name}: qkv has {C3} channels, expected 3*{heads}*{dim_head}")
    out = torch.empty((B, heads * dim_head, n), device=qkv.device, dtype=torch.float32)
    call(name, ptr(qkv), B, heads, dim_head, n, ptr(out), stream_ptr())
    return out


def linear_attention(qkv, heads, dim_head):
    """LinearAttention core (:245-258) on to_qkv's output."""
    return _attn("tvq_fe_linear_attention", qkv, heads, dim_head)


def linear_attention_fused(x, w_qkv, heads, dim_head):
    """to_qkv (1x1, no bias) + LinearAttention core in one kernel, bitwise equal to
    conv1d + linear_attention: the (B, 3 H dh, n) qkv tensor stays in LDS."""
    x, w = _c(x), _c(w_qkv)
    B, C, n = x.shape
    if w.shape[0] != 3 * heads * dim_head or w.shape[1] != C or w[0].numel() != C:
        raise ValueError(f"linear_attention_fused: weight {tuple(w.shape)} vs x {tuple(x.shape)}")
    kv = max(2 * 32 * (n + 1), 4 * 32 * 36)
    if (kv + 32 * 36 + C * n + 96 * C) * 4 > 160 * 1024 or dim_head != 32:
        # x and the head's weights do not fit beside q/k/v in LDS: the two-kernel HIP path
        return linear_attention(conv1d(x, w), heads, dim_head)
    out = torch.empty((B, heads * dim_head, n), device=x.device, dtype=torch.float32)
    call("tvq_fe_linear_attention_fused", ptr(x), B, C, n, ptr(w), heads, dim_head, ptr(out),
         stream_ptr())
    return out


def attention(qkv, heads, dim_head):
    """Attention core (:273-282) on to_qkv's output."""
    return _attn("tvq_fe_attention", qkv, heads, dim_head)


def cat_interp(a, b, length):
    """torch.cat((interp(a, length), interp(b, length)), 1), linear, align_corners=False
    (:434-452); b may be None (interpolate a alone, :495-497)."""
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
    return out
