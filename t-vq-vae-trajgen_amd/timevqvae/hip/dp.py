"""Data-parallel replica exchange (the reference itself runs one device,
scripts/train.py:33-43).

Per optimizer step every replica:
  * averages its flat gradient buffer over the ranks (one all-reduce per optimizer: the
    parameters are views into FusedAdamW's flat buffer, hip/optim.py);
  * ORs the layer-dropout gates (MAX), so every replica updates the same segments;
  * averages the BatchNorm running statistics (one all-reduce over a flat buffer that every
    running_mean / running_var is a view of).  DDP's `broadcast_buffers` copies rank 0's
    statistics into every replica before each forward; the mean keeps the replicas
    bitwise identical in the same way and is, for the running mean, exactly the update the
    single-process global batch would make (equal shard sizes).
The codebook EMA is NOT in that buffer: its statistics are summed before the EMA by the
reference's own sync_codebook hook (vq.py:155,229,234; hip/vq.py CodebookUpdate).
"""
import torch
import torch.distributed as dist
import torch.nn as nn


def batchnorm_modules(modules):
    """Every BatchNorm of `modules` that tracks running statistics, each once, in module
    order."""
    out, seen = [], set()
    for m in modules:
        for mod in m.modules():
            if (isinstance(mod, nn.modules.batchnorm._BatchNorm) and mod.track_running_stats
                    and id(mod) not in seen):
                seen.add(id(mod))
                out.append(mod)
    return out


def flatten_bn_buffers(modules):
    """Move the running_mean / running_var of every BatchNorm in `modules` into one flat
    fp32 buffer and make each buffer a view of it (the kernels update them in place through
    their addresses, so the views stay live).  Call after the modules are on their device;
    moving them again (module.to) re-allocates the buffers and detaches them from the flat
    one.  Returns the flat buffer, or None if there is no BatchNorm."""
    bns = batchnorm_modules(modules)
    if not bns:
        return None
    dev = bns[0].running_mean.device
    n = sum(b.running_mean.numel() + b.running_var.numel() for b in bns)
    flat = torch.empty(n, device=dev, dtype=torch.float32)
    off = 0
    with torch.no_grad():
        for b in bns:
            for name in ("running_mean", "running_var"):
                t = getattr(b, name)
                if t.device != dev or t.dtype != torch.float32:
                    raise ValueError("flatten_bn_buffers: running statistics must be fp32 on "
                                     "one device")
                k = t.numel()
                flat[off:off + k].copy_(t.reshape(-1))
                setattr(b, name, flat[off:off + k].view_as(t))
                off += k
    return flat


class ReplicaSync:
    """The exchange of one optimizer step over the default process group."""

    def __init__(self, world: int):
        self.world = int(world)

    def gradients(self, opt):
        """Mean of the flat gradients; layer-dropout gates OR-ed (MAX)."""
        if self.world <= 1:
            return
        dist.all_reduce(opt.flat_grad)
        opt.flat_grad.mul_(1.0 / self.world)
        if getattr(opt, "has_gates", False):
            dist.all_reduce(opt.gates, op=dist.ReduceOp.MAX)

    def buffers(self, flat):
        """Mean of the flat BatchNorm running statistics."""
        if self.world <= 1 or flat is None:
            return
        dist.all_reduce(flat)
        flat.mul_(1.0 / self.world)
