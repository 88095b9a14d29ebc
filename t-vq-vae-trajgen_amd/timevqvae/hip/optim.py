"""Fused AdamW over one flat parameter buffer (torch.optim.AdamW semantics).

The optimizer re-binds every trainable parameter to a view of one contiguous fp32
buffer and every .grad to a view of one flat gradient buffer, so that
  * zero_grad is one memset, the DP gradient all-reduce is one collective,
  * the update is one kernel launch (tvq_adamw) for the whole model.
lr and the step counter live on the device ({lr, step}); schedulers keep working
through param_groups[0]['lr'].
"""
import torch

from . import streams
from ._native import call, ptr, stream_ptr


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        params = [p for p in params if p.requires_grad]
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        if len(self.param_groups) != 1:
            raise NotImplementedError("FusedAdamW supports one param group")
        ps = self.param_groups[0]["params"]
        dev = ps[0].device
        if any(p.device != dev or p.dtype != torch.float32 for p in ps):
            raise ValueError("FusedAdamW: all parameters must be fp32 on one device")
        n = sum(p.numel() for p in ps)
        self.numel = n
        self.flat = torch.empty(n, device=dev, dtype=torch.float32)
        self.flat_grad = torch.zeros(n, device=dev, dtype=torch.float32)
        self.exp_avg = torch.zeros(n, device=dev, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros(n, device=dev, dtype=torch.float32)
        self.lr_step = torch.tensor([lr, 0.0], device=dev, dtype=torch.float32)
        off = 0
        with torch.no_grad():
            for p in ps:
                k = p.numel()
                self.flat[off:off + k].copy_(p.reshape(-1))
                p.data = self.flat[off:off + k].view_as(p)
                p.grad = self.flat_grad[off:off + k].view_as(p)
                p._tvq_flat = True
                off += k

    def push_lr(self):
        """Write param_groups[0]['lr'] into the device {lr, step} pair (for graph replays,
        whose captured update reads the lr from the device: step(lr_on_device=True))."""
        self.lr_step[0:1].fill_(float(self.param_groups[0]["lr"]))

    def zero_grad(self, set_to_none: bool = False):
        # gradients accumulate in place into the flat buffer views
        self.flat_grad.zero_()

    @torch.no_grad()
    def step(self, closure=None, lr_on_device=False):
        loss = closure() if closure is not None else None
        streams.join(self.flat.device, backward_done=True)  # grads written on side streams
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        s = stream_ptr()
        call("tvq_adamw_begin", ptr(self.lr_step), -1.0 if lr_on_device else float(g["lr"]), s)
        call("tvq_adamw", ptr(self.flat), ptr(self.flat_grad), ptr(self.exp_avg),
             ptr(self.exp_avg_sq), self.numel, ptr(self.lr_step), float(b1), float(b2),
             float(g["eps"]), float(g["weight_decay"]), s)
        return loss
