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
