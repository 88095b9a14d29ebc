"""Deferred, grouped weight gradients (tvq_wgrad_group).

nn.Linear's backward is dX = dY W (needed at once: the backward chain continues through
it) and dW = dY^T X (read by nothing until the optimizer step).  Inside a `grouped()`
scope, `weight_grad` records dW (+)= dY^T X instead of launching it; at the scope's exit
each stream's records go out as ONE grouped launch (+ one ordered slab sum) on the stream
that produced them.  For the LF prior that is 16 weight gradients (5.03 GFLOP) in one
launch that fills the chip, against 16 latency-bound split-K launch pairs.

Records keep their dY / X tensors alive until the flush is enqueued on their stream
(stream-ordered reuse afterwards, as for any tensor freed after its last kernel).  A
record whose output overlaps one already pending on its stream flushes the pending ones
first, so accumulations into one buffer keep their backward order.  The autograd engine
runs CUDA backward nodes on its device thread; the scope is process-global and the
issuing thread blocks in backward() meanwhile, so the records are complete at exit.
"""
import contextlib
import ctypes
import os

import torch

from ._native import call, ptr, value

ENABLED = True   # False: every weight gradient at once (tests)
_DEBUG = False   # print each launch's shapes

_pending = None  # (stream, tag) -> list of records while a scope is active
_tag = [None]


@contextlib.contextmanager
def tag(name):
    """Records of the Linear layers whose forward runs in the body form their own launch
    (e.g. one per prior): the launch plan is made per launch, so the grouping must not
    depend on the streams (a one-stream step puts both priors on one stream)."""
    prev = _tag[0]
    _tag[0] = name
    try:
        yield
    finally:
        _tag[0] = prev


def current_tag():
    return _tag[0]


@contextlib.contextmanager
def grouped():
    """Defer weight gradients issued in the body; flush them per stream at exit."""
    global _pending
    if _pending is not None or not ENABLED:
        yield
        return
    _pending = {}
    try:
        yield
    finally:
        pend, _pending = _pending, None
        for (st, _), recs in pend.items():
            if recs:
                with torch.cuda.stream(st):
                    launch(recs)


def launch(recs):
    """dW (+)= dY^T X for each record (dy, ldy, x, ldx, dw, ldw, M, N, K[, db]) in one
    tvq_wgrad_group_bias call on the current stream; a record's optional 10th entry is its
    bias gradient db (+)= the column sums of dY, taken in the same launch pair."""
    n = len(recs)
    dev = recs[0][0].device
    if _DEBUG:
        print("tvq_wgrad_group", torch.cuda.current_stream().stream_id,
              [(r[6], r[7], r[8]) for r in recs], flush=True)
    I64s = ctypes.c_int64 * n
    Ps = ctypes.c_void_p * n
    M, N, K = I64s(*[r[6] for r in recs]), I64s(*[r[7] for r in recs]), I64s(*[r[8] for r in recs])
    wsz = value("tvq_wgrad_group_workspace", n, ctypes.addressof(M), ctypes.addressof(N),
                ctypes.addressof(K))
    ws = torch.empty(wsz, device=dev, dtype=torch.float32) if wsz > 0 else None
    dy, x, dw = Ps(*[ptr(r[0]) for r in recs]), Ps(*[ptr(r[2]) for r in recs]), Ps(*[ptr(r[4]) for r in recs])
    ldy, ldx, ldw = I64s(*[r[1] for r in recs]), I64s(*[r[3] for r in recs]), I64s(*[r[5] for r in recs])
    dbs = [r[9] if len(r) > 9 else None for r in recs]
    db = Ps(*[ptr(t) if t is not None else None for t in dbs])
    call("tvq_wgrad_group_bias", n, ctypes.addressof(dy), ctypes.addressof(ldy), ctypes.addressof(x),
         ctypes.addressof(ldx), ctypes.addressof(dw), ctypes.addressof(ldw),
         ctypes.addressof(db) if any(t is not None for t in dbs) else None, ctypes.addressof(M),
         ctypes.addressof(N), ctypes.addressof(K), 1, ptr(ws),
         torch.cuda.current_stream().cuda_stream)


def _span(t, rows, ld, cols):
    a = t.data_ptr()
    return a, a + 4 * ((rows - 1) * ld + cols)


def _spans(r):
    out = [_span(r[4], r[6], r[5], r[7])]
    if len(r) > 9 and r[9] is not None:
        out.append(_span(r[9], 1, r[6], r[6]))
    return out


def defer(dy, ldy, x, ldx, dw, ldw, M, N, K, tag=None, db=None):
    """Record dW[m*ldw + n] += sum_k dY[k*ldy + m] X[k*ldx + n] (m < M, n < N, k < K)
    -- and, with `db` (a contiguous flat-gradient view of M floats), db[m] += sum_k
    dY[k*ldy + m] -- when a grouped() scope is active (returns True); else returns False
    and the caller launches it.  The flat-gradient views must not be read or written by
    anything else before the scope's exit (Linear weight / bias gradients: read by the
    optimizer only).  `tag`: the current_tag() of the layer's forward (records group per
    stream and tag)."""
    if _pending is None:
        return False
    rec = (dy, ldy, x, ldx, dw, ldw, M, N, K, db)
    st = torch.cuda.current_stream()
    recs = _pending.setdefault((st, tag), [])
    mine = _spans(rec)
    for other in [v for (s_, _), v in _pending.items() if s_ == st]:
        if any(lo < h and l < hi for r in other for l, h in _spans(r) for lo, hi in mine):
            launch(other)  # same output: keep the accumulation order
            other.clear()
    recs.append(rec)
    return True
