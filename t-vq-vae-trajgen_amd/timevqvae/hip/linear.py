"""Dense GEMM ops (nn.Linear over the last dim) on the HIP path."""
import torch

from . import streams, wgrad
from ._native import call, grad_sink, ptr, stream_ptr, value


def gemm(A, sam, sak, B, sbk, sbn, M, N, K, out=None, ldc=None, alpha=1.0, bias=None, R=None,
         ldr=0, rmod=0, act=0, pre=None, accumulate=False, gate=None):
    dev = A.device
    if out is None:
        out = torch.empty((M, N), device=dev, dtype=torch.float32)
        ldc = N
    wsz = value("tvq_gemm_workspace", M, N, K)
    ws = torch.empty(wsz, device=dev, dtype=torch.float32) if wsz > 0 else None
    call("tvq_gemm", ptr(A), sam, sak, ptr(B), sbk, sbn, ptr(out), ldc, M, N, K, float(alpha),
         ptr(bias), ptr(R), ldr, int(rmod), int(act), ptr(pre), int(bool(accumulate)), ptr(gate),
         ptr(ws), stream_ptr())
    return out


def _bias_grad_rows(g2, sink=None):
    """Column sums of a row-major (M, N) gradient: returned, or accumulated into `sink`."""
    M, N = g2.shape
    if sink is not None:  # into the flat gradient: off the critical path
        with streams.offload(g2):
            ws = torch.empty(value("tvq_channel_sum_workspace", M, N, 1), device=g2.device)
            call("tvq_channel_sum", ptr(g2), M, N, 1, ptr(sink), 1, ptr(ws), stream_ptr())
        return None
    out = torch.empty(N, device=g2.device, dtype=torch.float32)
    ws = torch.empty(value("tvq_channel_sum_workspace", M, N, 1), device=g2.device)
    call("tvq_channel_sum", ptr(g2), M, N, 1, ptr(out), 0, ptr(ws), stream_ptr())
    return out


def weight_grad(g, x2, w_param, M, N, K, tag=None, b_param=None):
    """dW = g^T x (N x K): accumulated into the flat grad view when available (deferred to
    the grouped launch inside a wgrad.grouped() scope; `tag`: the forward's wgrad tag).
    With `b_param`: returns (dW, db), db = the column sums of g; inside a grouped() scope,
    with both flat-gradient views available, db rides in the same grouped launch."""
    sink = grad_sink(w_param)
    if b_param is not None:
        bsink = grad_sink(b_param)
        if sink is not None and bsink is not None and wgrad.defer(
                g, N, x2, K, sink, K, N, K, M, tag, db=bsink):
            return None, None
        return weight_grad(g, x2, w_param, M, N, K, tag), _bias_grad_rows(g, bsink)
    if sink is not None:  # into the flat gradient: off the critical path
        if wgrad.defer(g, N, x2, K, sink, K, N, K, M, tag):  # grouped at the backward's end
            return None
        with streams.offload(g, x2):
            gemm(g, 1, N, x2, K, 1, N, K, M, out=sink, ldc=K, accumulate=True)
        return None
    return gemm(g, 1, N, x2, K, 1, N, K, M)


def scale_by(x, s):
    """x * s[0] (s: a one-element device tensor) in one kernel."""
    x = x.contiguous()
    y = torch.empty_like(x)
    call("tvq_scale_by", ptr(x), x.numel(), ptr(s), ptr(y), stream_ptr())
    return y


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, residual, gate):
        shp = x.shape
        K = shp[-1]
        N = w.shape[0]
        x2 = x.reshape(-1, K).contiguous()
        w = w.contiguous()
        M = x2.shape[0]
        R = residual.reshape(M, N).contiguous() if residual is not None else None
        y = gemm(x2, K, 1, w, 1, K, M, N, K, bias=b, R=R, ldr=N, gate=gate)
        ctx.save_for_backward(x2, w)
        ctx.has = (b is not None, residual is not None)
        ctx.shp = shp
        ctx.params = (w, b)
        ctx.wg_tag = wgrad.current_tag()
        ctx.gate = gate
        return y.reshape(*shp[:-1], N)

    @staticmethod
    def backward(ctx, gy):
        x2, w = ctx.saved_tensors
        M, K = x2.shape
        N = w.shape[0]
        dres = gy if ctx.has[1] and ctx.needs_input_grad[3] else None
        # gated branch (layer dropout): the branch's gradient is gate * gy
        g = scale_by(gy, ctx.gate) if ctx.gate is not None else gy
        g = g.reshape(M, N).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = gemm(g, N, 1, w, K, 1, M, K, N).reshape(ctx.shp)
        if ctx.needs_input_grad[1] and ctx.has[0] and ctx.needs_input_grad[2]:
            dw, db = weight_grad(g, x2, ctx.params[0], M, N, K, ctx.wg_tag, ctx.params[1])
        else:
            if ctx.needs_input_grad[1]:
                dw = weight_grad(g, x2, ctx.params[0], M, N, K, ctx.wg_tag)
            if ctx.has[0] and ctx.needs_input_grad[2]:
                db = _bias_grad_rows(g, grad_sink(ctx.params[1]))
        return dx, dw, db, dres, None


class _LinearSelfRes(torch.autograd.Function):
    """y = x + x W^T + b (vq_vae.py:263 `out + self.linear(out)`, W square): x has one
    autograd consumer and dx = dy W + dy comes out of one GEMM (residual epilogue)."""

    @staticmethod
    def forward(ctx, x, w, b):
        shp = x.shape
        K = shp[-1]
        x2 = x.reshape(-1, K).contiguous()
        M = x2.shape[0]
        y = gemm(x2, K, 1, w.contiguous(), 1, K, M, K, K, bias=b, R=x2, ldr=K)
        ctx.save_for_backward(x2, w)
        ctx.params = (w, b)
        ctx.wg_tag = wgrad.current_tag()
        ctx.shp = shp
        return y.reshape(shp)

    @staticmethod
    def backward(ctx, gy):
        x2, w = ctx.saved_tensors
        M, K = x2.shape
        g = gy.reshape(M, K).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = gemm(g, K, 1, w.contiguous(), K, 1, M, K, K, R=g, ldr=K).reshape(ctx.shp)
        if ctx.needs_input_grad[1] and ctx.params[1] is not None and ctx.needs_input_grad[2]:
            dw, db = weight_grad(g, x2, ctx.params[0], M, K, K, ctx.wg_tag, ctx.params[1])
        else:
            if ctx.needs_input_grad[1]:
                dw = weight_grad(g, x2, ctx.params[0], M, K, K, ctx.wg_tag)
            if ctx.params[1] is not None and ctx.needs_input_grad[2]:
                db = _bias_grad_rows(g, grad_sink(ctx.params[1]))
        return dx, dw, db


def linear(x, weight, bias=None, residual=None, gate=None):
    """residual + gate * (x @ weight^T + bias) over the last dim (nn.Linear; vq_vae.py:255,263;
    `gate`: optional one-element device tensor, the x-transformers layer-dropout keep flag)."""
    if residual is x and gate is None and weight.shape[0] == weight.shape[1]:
        return _LinearSelfRes.apply(x, weight, bias)
    return _Linear.apply(x, weight, bias, residual, gate)


class _WeightProduct(torch.autograd.Function):
    """W = W1 W2 for two Linears that meet without a nonlinearity between them (x W2^T W1^T =
    x (W1 W2)^T); backward dW1 = dW W2^T, dW2 = W1^T dW, accumulated into the flat-gradient
    sinks when they exist (tiny GEMMs)."""

    @staticmethod
    def forward(ctx, w1, w2):
        w1 = w1.contiguous()
        w2 = w2.contiguous()
        M, K = w1.shape
        N = w2.shape[1]
        ctx.save_for_backward(w1, w2)
        ctx.params = (w1, w2)
        return gemm(w1, K, 1, w2, N, 1, M, N, K)

    @staticmethod
    def backward(ctx, g):
        w1, w2 = ctx.saved_tensors
        M, K = w1.shape
        N = w2.shape[1]
        g = g.contiguous()
        out = [None, None]
        if ctx.needs_input_grad[0]:
            sk = grad_sink(ctx.params[0])
            d = sk if sk is not None else torch.empty_like(w1)
            gemm(g, N, 1, w2, 1, N, M, K, N, out=d, ldc=K, accumulate=sk is not None)
            out[0] = None if sk is not None else d
        if ctx.needs_input_grad[1]:
            sk = grad_sink(ctx.params[1])
            d = sk if sk is not None else torch.empty_like(w2)
            gemm(w1, 1, K, g, N, 1, K, N, M, out=d, ldc=N, accumulate=sk is not None)
            out[1] = None if sk is not None else d
        return out[0], out[1]


def weight_product(w1, w2):
    """w1 @ w2 with autograd into w1 / w2 (their flat-gradient sinks when present)."""
    return _WeightProduct.apply(w1, w2)
