"""Fused AdamW over one flat parameter buffer (torch.optim.AdamW semantics).

The optimizer re-binds every trainable parameter to a view of one contiguous fp32
buffer and every .grad to a view of one flat gradient buffer, so that
  * zero_grad is one memset, the DP gradient all-reduce is one collective,
  * the update is one kernel launch (tvq_adamw) for the whole model.
lr lives on the device ({lr, step}); schedulers keep working through
param_groups[0]['lr'].

Skipped parameters.  torch.optim.AdamW leaves a parameter whose .grad is None alone
(no weight decay, no moment update, its own state['step'] not advanced); under
Lightning's zero_grad(set_to_none=True) that is every parameter of an x-transformers
branch that layer dropout skipped this step (bidirectional_transformer.py:104-108).
Each parameter is one segment of the flat buffer with its own step count; a
parameter tagged `_tvq_gate = (module, i)` (set by the transformer Encoder) is updated
only when `module._touched[i]` is non-zero after the step's forward passes.
"""
import ctypes

import torch

from . import streams
from ._native import call, ptr, stream_ptr, value

_grad_epoch = [0]


def grad_epoch() -> int:
    """Incremented by every FusedAdamW.zero_grad: a module that records which of its
    branches ran (Encoder._touched) starts a new record on the first forward of an epoch."""
    return _grad_epoch[0]


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
        chunk = int(value("tvq_adamw_chunk"))
        chunks, gate_ptrs = [], []
        self._gate_refs = []  # keeps every gate tensor's storage alive
        # (segment, owner module, index, address at construction): gather_gates checks that
        # no owner's `_touched` buffer moved (module.to / _apply / buffer replacement) before
        # the gate kernel dereferences the recorded addresses.  A deepcopy'd parameter loses
        # its `_tvq_gate` attribute and is updated ungated (plain AdamW).
        self._gate_owners = []
        off = 0
        with torch.no_grad():
            for s, p in enumerate(ps):
                k = p.numel()
                self.flat[off:off + k].copy_(p.reshape(-1))
                p.data = self.flat[off:off + k].view_as(p)
                p.grad = self.flat_grad[off:off + k].view_as(p)
                p._tvq_flat = True
                for c in range(0, k, chunk):
                    chunks.append((off + c, min(chunk, k - c), s))
                gate = getattr(p, "_tvq_gate", None)
                if gate is not None:
                    owner, i = gate
                    t = owner._touched
                    if t.device != dev:
                        raise ValueError("FusedAdamW: a gate buffer is not on the parameters' "
                                         "device (build the optimizer after .to(device))")
                    self._gate_refs.append(t)
                    self._gate_owners.append((s, owner, i, t.data_ptr()))
                    gate_ptrs.append(t.data_ptr() + 4 * i)
                else:
                    gate_ptrs.append(0)
                off += k
        self.nseg = len(ps)
        self.chunks = torch.tensor(chunks, dtype=torch.int64, device=dev).reshape(-1)
        self.nchunks = len(chunks)
        self.gate_ptrs = torch.tensor(gate_ptrs, dtype=torch.int64, device=dev)
        self.gates = torch.ones(self.nseg, device=dev, dtype=torch.float32)
        self.seg_step = torch.zeros(self.nseg, device=dev, dtype=torch.float32)
        self.has_gates = any(gate_ptrs)
        # zero_after_step (opt-in, a fixed zero_grad -> backward -> step loop such as
        # bench.JointTrainer's replayed step): the update zeroes each gradient value after
        # reading it, and the next zero_grad() -- when nothing else ran in between -- has
        # nothing left to fill.  .grad then reads 0 after step() (torch keeps it until
        # zero_grad), so it is off by default.
        self.zero_after_step = False
        self._clean = False

    def push_lr(self, other=None):
        """Write param_groups[0]['lr'] into the device {lr, step} pair (for graph replays,
        whose captured update reads the lr from the device: step(lr_on_device=True));
        `other`: a second FusedAdamW whose lr goes in the same launch."""
        call("tvq_fill2", ptr(self.lr_step), float(self.param_groups[0]["lr"]),
             ptr(other.lr_step) if other is not None else None,
             float(other.param_groups[0]["lr"]) if other is not None else 0.0, stream_ptr())

    def zero_grad(self, set_to_none: bool = False):
        # gradients accumulate in place into the flat buffer views
        _grad_epoch[0] += 1
        if self.zero_after_step and self._clean:
            self._clean = False  # zeroed by the last step()'s update
            return
        self._clean = False
        call("tvq_fill", ptr(self.flat_grad), self.flat_grad.numel(), 0.0, stream_ptr())

    def gather_gates(self):
        """gates[s] <- whether segment s's gated branch ran this step (after the forward
        passes; under DP the trainer then all-reduces `gates` with MAX)."""
        if self.has_gates:
            self._check_gate_buffers()
            call("tvq_adamw_gates", ptr(self.gate_ptrs), self.nseg, ptr(self.gates), stream_ptr())

    def _check_gate_buffers(self):
        moved = [(seg, o, i) for seg, o, i, a in self._gate_owners if o._touched.data_ptr() != a]
        if not moved:
            return
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("FusedAdamW: a layer-dropout gate buffer moved since the optimizer "
                               "was built; re-run one eager step before capturing")
        ptrs = self.gate_ptrs.cpu()
        for seg, o, i in moved:
            t = o._touched
            if t.device != self.flat.device:
                raise ValueError("FusedAdamW: a gate buffer left the parameters' device")
            ptrs[seg] = t.data_ptr() + 4 * i
        self.gate_ptrs.copy_(ptrs)
        self._gate_refs = [o._touched for _, o, _, _ in self._gate_owners]
        self._gate_owners = [(seg, o, i, o._touched.data_ptr()) for seg, o, i, _ in self._gate_owners]

    @torch.no_grad()
    def step(self, closure=None, lr_on_device=False, gates_ready=False):
        loss = closure() if closure is not None else None
        streams.join(self.flat.device, backward_done=True)  # grads written on side streams
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        s = stream_ptr()
        if not gates_ready:
            self.gather_gates()
        call("tvq_adamw_begin", ptr(self.lr_step), -1.0 if lr_on_device else float(g["lr"]),
             ptr(self.gates), ptr(self.seg_step), self.nseg, s)
        call("tvq_adamw_zero", ptr(self.flat), ptr(self.flat_grad), ptr(self.exp_avg),
             ptr(self.exp_avg_sq), ptr(self.chunks), self.nchunks, ptr(self.lr_step),
             ptr(self.gates), ptr(self.seg_step), float(b1), float(b2), float(g["eps"]),
             float(g["weight_decay"]), int(self.zero_after_step), s)
        self._clean = self.zero_after_step
        return loss


@torch.no_grad()
def step_pair(a: "FusedAdamW", b: "FusedAdamW", lr_on_device=False, gates_ready=False):
    """a.step(); b.step() -- the same arithmetic -- as two launches instead of four
    (tvq_adamw2: both optimizers' step counts, then both updates); both zero the gradients
    they read when their zero_after_step is set (it must agree)."""
    if a.zero_after_step != b.zero_after_step:
        raise ValueError("step_pair: zero_after_step differs")
    streams.join(a.flat.device, backward_done=True)
    if not gates_ready:
        a.gather_gates()
        b.gather_gates()
    P2 = ctypes.c_void_p * 2
    I2 = ctypes.c_int64 * 2
    F2 = ctypes.c_float * 2
    opts = (a, b)
    gs = [o.param_groups[0] for o in opts]
    # every host array is kept in `keep` until the call returns (ctypes passes addresses)
    keep = [P2(*[ptr(o.flat) for o in opts]), P2(*[ptr(o.flat_grad) for o in opts]),
            P2(*[ptr(o.exp_avg) for o in opts]), P2(*[ptr(o.exp_avg_sq) for o in opts]),
            P2(*[ptr(o.chunks) for o in opts]), I2(a.nchunks, b.nchunks),
            P2(*[ptr(o.lr_step) for o in opts]),
            F2(*[-1.0 if lr_on_device else float(g["lr"]) for g in gs]),
            P2(*[ptr(o.gates) for o in opts]), P2(*[ptr(o.seg_step) for o in opts]),
            I2(a.nseg, b.nseg), F2(*[g["betas"][0] for g in gs]),
            F2(*[g["betas"][1] for g in gs]), F2(*[g["eps"] for g in gs]),
            F2(*[g["weight_decay"] for g in gs])]
    call("tvq_adamw2", *[ctypes.addressof(k) for k in keep], int(a.zero_after_step),
         stream_ptr())
    a._clean = a.zero_after_step
    b._clean = b.zero_after_step
