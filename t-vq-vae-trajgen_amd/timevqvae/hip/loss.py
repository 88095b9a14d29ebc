"""Reconstruction losses on the HIP path (stage1.py:129-135)."""
import torch

from ._native import call, ptr, stream_ptr, value

_KIND = {"mse": 0, "l1": 1}


class _Loss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inp, target, kind):
        a = inp.contiguous()
        b = target.contiguous()
        n = a.numel()
        out = torch.empty((), device=a.device, dtype=torch.float32)
        ws = torch.empty(value("tvq_loss_workspace", n), device=a.device, dtype=torch.float32)
        call("tvq_loss_fwd", ptr(a), ptr(b), n, kind, ptr(out), ptr(ws), stream_ptr())
        ctx.save_for_backward(a, b)
        ctx.kind = kind
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        dt = torch.empty_like(b)
        call("tvq_loss_bwd", ptr(a), ptr(b), a.numel(), ctx.kind, ptr(g), ptr(dt), stream_ptr())
        di = -dt if ctx.needs_input_grad[0] else None
        return di, dt if ctx.needs_input_grad[1] else None, None


def mse_loss(inp, target):
    return _Loss.apply(inp, target, 0)


def l1_loss(inp, target):
    return _Loss.apply(inp, target, 1)


def _flat_same(ts):
    n = ts[0].numel()
    return all(t.is_cuda and t.dtype == torch.float32 and t.numel() == n and t.is_contiguous()
               for t in ts)


class _Add2(torch.autograd.Function):
    """a + b (same shape) as one tvq_sum4 launch; the backward passes the gradient to both
    without a kernel (MaskGIT's mask_pred_loss_l + mask_pred_loss_h, maskgit.py:192)."""

    @staticmethod
    def forward(ctx, a, b):
        out = torch.empty_like(a)
        call("tvq_sum4", ptr(a), ptr(b), None, None, ptr(out), None, a.numel(), stream_ptr())
        return out

    @staticmethod
    def backward(ctx, g):
        return g, g


def add_losses(a, b):
    if not _flat_same((a, b)) or a.shape != b.shape:
        return a + b
    return _Add2.apply(a, b)


@torch.no_grad()
def loss_sums(rl, rh, vl, vh):
    """((rl + rh) + vl) + vh and rl + rh -- the logged totals of stage1.py:170-198 -- in one
    tvq_sum4 launch (no autograd: the bands were backpropagated from their own roots)."""
    ts = (rl, rh, vl, vh)
    if not _flat_same(ts):
        return ((rl + rh) + vl) + vh, rl + rh
    out, ab = torch.empty_like(vl), torch.empty_like(rl)  # shapes of the broadcast sums
    call("tvq_sum4", ptr(rl), ptr(rh), ptr(vl.reshape(rl.shape)), ptr(vh.reshape(rl.shape)),
         ptr(out), ptr(ab), rl.numel(), stream_ptr())
    return out, ab
