"""Branch concurrency on a second HIP stream.

The LF and HF branches of Stage1 (encoder -> VQ -> decoder -> loss) and of MaskGIT
(frozen encoders, the two bidirectional transformers) are independent chains of small
kernels.  Each kernel on this path is a few microseconds, so a single in-order stream
spends most of a step in kernel ramp-up/drain; issuing the HF chain on a side stream
lets the two chains overlap.  Autograd replays each backward node on the stream its
forward ran on, so the backward overlaps the same way.  Under hipGraph capture the
fork/join become graph edges and the branches are parallel graph nodes.

Concurrency is opt-in per region: `branch()` and `offload()` fork only inside
`concurrent()` (the training step of a trainer: forward + backward), and leaving the
outermost region joins every stream, so the modules used on their own (tests, a
Lightning loop reading .grad after backward) stay plain single-stream code.

`branch(device, key)` forks side stream `key` of the current stream; the branch's
`join()` makes the parent wait for it before the parent reads the branch's results
(end of a forward).  `join(backward_done=True)` makes the current stream wait for
every stream used in the region; it runs before anything reads gradients (region exit,
optimizer step, DP all-reduce): the flat-gradient sinks are written by backward
kernels on several streams, which the autograd engine does not synchronise (it only
syncs AccumulateGrad leaves).

Measured on MI355X (bench.py, config B, hipGraph): one stream 14.4 ms/step; LF||HF
branches 10.8; stage1 || stage2 (bench.JointTrainer) with stage1's LF||HF: 8.1.
Fine-grained forks (every weight gradient or codebook statistic on an aux stream,
`offload`) cost more in graph edges than they hide (+1 to +3 ms), so they are off
unless OFFLOAD names them.
"""
import contextlib
import os

import torch

ENABLED = True  # False (tests): one stream
# offload classes: "grad" (weight/bias gradients into the flat sinks), "vq" (codebook
# statistics + EMA).  Each offload is a fork + join edge in the captured graph, which
# costs more than a small kernel it takes off the critical path, so the default is none.
OFFLOAD = set()
# branch keys to run inline instead (experiments: "hf", "stage2")
INLINE = set()

_side = {}      # (device index, parent stream id, key) -> side stream
_used = {}      # parent stream id -> side streams forked from it since the last full join
_fences = {}    # key -> event: in-place buffer updates issued on an offload stream


_region = [0]
_depth = [0]    # branch nesting level of the code being issued


@contextlib.contextmanager
def concurrent():
    """Region in which branch()/offload() run on their own streams; the outermost exit
    joins them all (after the backward, so weight gradients are complete)."""
    _region[0] += 1
    try:
        yield
    finally:
        _region[0] -= 1
        if _region[0] == 0:
            join(backward_done=True)


def active():
    return ENABLED and _region[0] > 0


def side_stream(parent, key):
    k = (parent.device.index, parent.stream_id, key)
    s = _side.get(k)
    if s is None:
        s = torch.cuda.Stream(device=parent.device)
        _side[k] = s
    return s


def _tensors(obj):
    if isinstance(obj, torch.Tensor):
        yield obj
    elif isinstance(obj, dict):
        for v in obj.values():
            yield from _tensors(v)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            yield from _tensors(v)


class _Branch:
    def __init__(self, device, stream, main):
        self.device, self.stream, self.main = device, stream, main

    def inputs(self, *objs):
        """Tensors made on the parent stream and read on the branch."""
        if self.stream is not None:
            for t in _tensors(objs):
                if t.is_cuda:
                    t.record_stream(self.stream)

    def outputs(self, *objs):
        """Tensors made on the branch and read on the parent stream after join()."""
        if self.stream is not None:
            for t in _tensors(objs):
                if t.is_cuda:
                    t.record_stream(self.main)

    def join(self):
        """The parent stream waits for the work issued on this branch so far."""
        if self.stream is not None:
            self.main.wait_stream(self.stream)


@contextlib.contextmanager
def branch(device, key="hf", enabled=True):
    """Run the body on side stream `key` of the current stream (forked off it)."""
    if (not (active() and enabled) or key in INLINE or _depth[0] > 0
            or torch.device(device).type != "cuda"):
        # nested branches run inline: any dependency edge between two forked streams
        # (a fork off a forked stream, or a root fork that also waits on another branch)
        # makes the ROCm 7.2 runtime segfault in hipStreamEndCapture (measured), so the
        # graph keeps to root -> branch -> root edges
        yield _Branch(device, None, None)
        return
    main = torch.cuda.current_stream(device)
    s = side_stream(main, key)
    s.wait_stream(main)
    _depth[0] += 1
    try:
        with torch.cuda.stream(s):
            yield _Branch(device, s, main)
    finally:
        _depth[0] -= 1
    _used.setdefault(main.stream_id, set()).add(s)


def join(device=None, backward_done=True):
    """The current stream waits for every stream used since the last join (branches,
    their backward kernels, offloads)."""
    if not _used:
        return
    cur = torch.cuda.current_stream(device)
    _fences.clear()  # every stream's work is now ordered before the current stream
    ss = set().union(*_used.values())
    _used.clear()
    for s in ss:
        if s != cur:
            cur.wait_stream(s)


_aux = {}  # (device index, stream id) -> auxiliary stream of that stream


def aux_stream(cur):
    key = (cur.device.index, cur.stream_id)
    s = _aux.get(key)
    if s is None:
        s = torch.cuda.Stream(device=cur.device)
        _aux[key] = s
    return s


@contextlib.contextmanager
def offload(*inputs, kind="grad"):
    """Run the body on the auxiliary stream of the current stream: work nothing on the
    critical path waits for (weight gradients, codebook statistics).  `inputs` are the
    tensors made on the current stream that the body reads.  The results are joined by
    the next join(backward_done=True)."""
    cur = torch.cuda.current_stream()
    if not (active() and kind in OFFLOAD):
        yield cur
        return
    s = aux_stream(cur)
    s.wait_stream(cur)
    for t in _tensors(inputs):
        if t is not None and t.is_cuda:
            t.record_stream(s)
    with torch.cuda.stream(s):
        yield s
    _used.setdefault(cur.stream_id, set()).add(s)


def fence(key):
    """Mark an in-place update of buffer `key` just issued on the current (offload)
    stream; the buffer's next reader calls wait_fence(key) first."""
    if active():
        ev = torch.cuda.Event()
        ev.record()
        _fences[key] = ev


def wait_fence(key):
    ev = _fences.get(key)
    if ev is not None:
        torch.cuda.current_stream().wait_event(ev)
