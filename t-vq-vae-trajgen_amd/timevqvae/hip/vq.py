"""VQ codebook ops on the HIP path (include/tvq.h §VQ codebook).

Replaces EuclideanCodebook.forward + the straight-through/commitment part of
VectorQuantize.forward (reference timevqvae/models/vq.py:197-251, 357-366):
  assign (L2 + argmin + gather, fp32 MFMA)  ->  per-code stats (deterministic)
  -> [optional all-reduce of the stats: sync_codebook, vq.py:229,234]
  -> EMA blend -> Laplace-normalised codebook + perplexity + commit loss.
"""
import contextlib

import torch

from . import rng, streams
from ._native import call, ptr, stream_ptr, value

_SVQ_SITE = 0x5F << 56  # noise stream of the stochastic assignment (svq_temp > 0); fixed, so
# module-construction site numbering (rng.new_site) is unchanged

_pending = None  # list of CodebookUpdate while a deferral scope is active


class CodebookUpdate:
    """An EMA codebook update whose per-batch statistics are computed but not yet applied.

    The forward outputs never read the updated codebook (quantize = E_old[idx]), so the
    update can move after the backward: `reduce()` runs the sync_codebook all-reduce of
    the statistics (eager, between captured graph segments) and `apply()` the EMA blend +
    Laplace-normalised codebook (capturable).
    """

    def __init__(self, cs_b, es_b, cluster_size, embed_avg, embed, decay, eps, sync):
        self.cs_b, self.es_b = cs_b, es_b
        self.cluster_size, self.embed_avg, self.embed = cluster_size, embed_avg, embed
        self.decay, self.eps, self.sync = decay, eps, sync
        self.K, self.D = embed.shape

    def reduce(self):
        if self.sync is not None:
            self.sync(self.cs_b)
            self.sync(self.es_b)

    def apply(self):
        s = stream_ptr()
        call("tvq_vq_ema", ptr(self.cs_b), ptr(self.es_b), self.K, self.D, float(self.decay),
             ptr(self.cluster_size), ptr(self.embed_avg), s)
        call("tvq_vq_finalize", ptr(self.cluster_size), ptr(self.embed_avg), self.K, self.D,
             float(self.eps), ptr(self.embed), None, 0, None, None, 0, None, s)


@contextlib.contextmanager
def deferred_codebook_updates():
    """Collect the EMA codebook updates of the passes run inside the scope instead of
    applying them; yields the list of CodebookUpdate (reduce() then apply() each)."""
    global _pending
    prev, _pending = _pending, []
    try:
        yield _pending
    finally:
        _pending = prev


_indices_only = [False]


@contextlib.contextmanager
def indices_only():
    """Eval codebook passes in the body skip the per-code counts and the perplexity (their
    group-by and reductions): for callers that read only the indices, such as MaskGIT's
    frozen tokenizer (maskgit.py:117-134 discards the perplexity).  Training passes are
    unaffected (their EMA needs the statistics)."""
    prev = _indices_only[0]
    _indices_only[0] = True
    try:
        yield
    finally:
        _indices_only[0] = prev


def _same_dense_layout(a, b):
    return a.shape == b.shape and a.stride() == b.stride()


def _check_dense(x):
    order = sorted(range(x.dim()), key=lambda i: -x.stride(i))
    if not x.permute(order).is_contiguous():
        raise ValueError("tvq VQ: input must be a dense (possibly permuted) tensor")


def vq_codebook_pass(x, embed, cluster_size, embed_avg, *, straight_through, ema, decay, eps,
                     sync=None, svq_temp=None, gumbel=None):
    """One codebook pass over x (B,N,D).

    svq_temp > 0: stochastic assignment idx ~ Categorical(softmax(dist / svq_temp))
    (vq.py:51-56, 216-222), drawn on the device by Gumbel-max; `gumbel` (M, K) injects the
    noise (tests), otherwise it comes from the device seed (hip/rng.py).

    Returns (out, idx, commit, perplexity, counts):
      out   = x + (E[idx]-x) if straight_through else E[idx]  (pre-update codebook)
      idx   = int64 (B,N);  commit = mean((out-x)^2) (0-dim) if straight_through else None
      perplexity 0-dim;     counts = int32 (K,)
    With ema=True the buffers cluster_size/embed_avg/embed are updated in place.
    """
    B, N, D = x.shape
    K = embed.shape[0]
    M = B * N
    _check_dense(x)
    dev = x.device
    streams.wait_fence(embed.data_ptr())  # an EMA update of this codebook may be in flight
    s = stream_ptr()
    ee = torch.empty(K, device=dev, dtype=torch.float32)
    call("tvq_vq_sqnorm", ptr(embed), K, D, ptr(ee), s)
    out = torch.empty_like(x)
    assert _same_dense_layout(out, x)
    idx = torch.empty((B, N), device=dev, dtype=torch.long)
    idx32 = torch.empty(M, device=dev, dtype=torch.int32)
    nb = value("tvq_vq_assign_nblocks", M)
    partial = torch.empty(nb, device=dev, dtype=torch.float32) if straight_through else None
    sB, sN, sD = x.stride()
    # EMA statistics sum token rows per code: with an NCHW latent (sD > 1) the assign pass
    # also writes x token-major so that those sums read contiguous rows
    rows = (torch.empty((M, D), device=dev, dtype=torch.float32)
            if ema and straight_through and sD != 1 else None)
    seed, off = None, 0
    if svq_temp:
        if gumbel is not None and (gumbel.shape != (M, K) or not gumbel.is_contiguous()):
            raise ValueError("vq: injected gumbel noise must be a contiguous (M, K) tensor")
        seed = rng.seed_tensor(dev) if gumbel is None else None
        off = rng.call_offset(_SVQ_SITE) if gumbel is None else 0
    call("tvq_vq_assign_rows", ptr(x), B, N, D, sB, sN, sD, ptr(embed), ptr(ee), K,
         int(bool(straight_through)), float(svq_temp or 0.0), ptr(gumbel), ptr(seed), off,
         ptr(out), ptr(idx), ptr(idx32), ptr(partial), ptr(rows), s)
    commit = torch.empty((), device=dev, dtype=torch.float32) if straight_through else None
    # the commitment mean is read only by the loss report at the band's end (its gradient
    # does not need it): it joins the statistics' finish launch unless those are skipped or
    # offloaded to another stream (then it is finished here, on the current stream)
    late = not (_indices_only[0] and not ema) and "vq" not in streams.OFFLOAD
    if straight_through and not late:
        call("tvq_vq_finalize", None, None, K, D, float(eps), None, None, M, None, ptr(partial),
             nb, ptr(commit), s)
    # per-code statistics, EMA and perplexity: nothing downstream of the quantised output
    # waits for them (inside streams.concurrent() they run on the aux stream; the region's
    # join completes them before anyone reads the perplexity or the codebook)
    if _indices_only[0] and not ema:
        return out, idx, commit, None, None
    src = rows.view(1, M, D) if rows is not None else x
    cm = (partial, nb, commit) if straight_through and late else (None, 0, None)
    with streams.offload(src, idx32, kind="vq"):
        counts, perp = _codebook_stats(src, idx32, embed, cluster_size, embed_avg, ema, decay,
                                       eps, sync, cm)
    return out, idx, commit, perp, counts


def _codebook_stats(x, idx32, embed, cluster_size, embed_avg, ema, decay, eps, sync,
                    cm=(None, 0, None)):
    """cm = (commit partials, their count, commit): the commitment mean, finished by the
    same vq_finalize launch as the perplexity."""
    cpart, nb, commit = cm
    B, N, D = x.shape
    K = embed.shape[0]
    M = B * N
    dev = x.device
    sB, sN, sD = x.stride()
    s = stream_ptr()
    counts = torch.empty(K, device=dev, dtype=torch.int32)
    cs_b = torch.empty(K, device=dev, dtype=torch.float32)
    es_b = torch.empty((K, D), device=dev, dtype=torch.float32) if ema else None
    ws = torch.empty(value("tvq_vq_stats_workspace", M, K), device=dev, dtype=torch.int32)
    call("tvq_vq_stats", ptr(x), B, N, D, sB, sN, sD, ptr(idx32), K, ptr(counts), ptr(cs_b),
         ptr(es_b), ptr(ws), s)
    perp = torch.empty((), device=dev, dtype=torch.float32)
    if ema and _pending is not None:
        _pending.append(CodebookUpdate(cs_b, es_b, cluster_size, embed_avg, embed, decay, eps, sync))
        call("tvq_vq_finalize", None, None, K, D, float(eps), None, ptr(counts), M, ptr(perp),
             ptr(cpart), nb, ptr(commit), s)
    elif ema:
        if sync is not None:
            sync(cs_b)
            sync(es_b)
            s = stream_ptr()
        call("tvq_vq_ema", ptr(cs_b), ptr(es_b), K, D, float(decay), ptr(cluster_size),
             ptr(embed_avg), s)
        call("tvq_vq_finalize", ptr(cluster_size), ptr(embed_avg), K, D, float(eps), ptr(embed),
             ptr(counts), M, ptr(perp), ptr(cpart), nb, ptr(commit), s)
        streams.fence(embed.data_ptr())
    else:
        call("tvq_vq_finalize", None, None, K, D, float(eps), None, ptr(counts), M, ptr(perp),
             ptr(cpart), nb, ptr(commit), s)
    return counts, perp


class _VQStraightThrough(torch.autograd.Function):
    """Training pass: forward = codebook pass with EMA; backward of vq.py:358,364."""

    @staticmethod
    def forward(ctx, x, embed, cluster_size, embed_avg, ema, decay, eps, sync, svq_temp):
        out, idx, commit, perp, _ = vq_codebook_pass(
            x, embed, cluster_size, embed_avg, straight_through=True, ema=ema, decay=decay,
            eps=eps, sync=sync, svq_temp=svq_temp)
        ctx.save_for_backward(x, out)
        ctx.mark_non_differentiable(idx, perp)
        ctx.set_materialize_grads(False)  # no zero-filled grads for idx / perp (None handled)
        return out, idx, commit, perp

    @staticmethod
    def backward(ctx, g_out, g_idx, g_commit, g_perp):
        x, out = ctx.saved_tensors
        if g_out is None:
            g_out = torch.zeros_like(x)
        elif not _same_dense_layout(g_out, x):
            g = torch.empty_like(x)
            g.copy_(g_out)
            g_out = g
        dx = torch.empty_like(x)
        gc = g_commit.contiguous() if g_commit is not None else None
        call("tvq_vq_backward", ptr(x), ptr(out), ptr(g_out), ptr(gc), x.numel(), x.numel(),
             ptr(dx), stream_ptr())
        return dx, None, None, None, None, None, None, None, None


def vq_train(x, embed, cluster_size, embed_avg, *, ema, decay, eps, sync=None, svq_temp=None):
    """Training-mode VQ with straight-through gradient. Returns (out, idx, commit, perp)."""
    return _VQStraightThrough.apply(x, embed, cluster_size, embed_avg, ema, decay, eps, sync,
                                    svq_temp)
