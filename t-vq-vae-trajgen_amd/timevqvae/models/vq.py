"""EMA vector quantiser — same API as the reference timevqvae/models/vq.py.

`VectorQuantize(dim, codebook_size, ...)` and its `_codebook` (EuclideanCodebook)
keep the reference constructor signature, buffer names
(`_codebook.{initted,cluster_size,embed_avg,embed}`) and forward contract
`forward(x (B,N,D), svq_temp=None) -> (quantize, embed_ind, vq_loss, perplexity)`
(vq.py:255-407).  The arithmetic runs in libtvq_hip.so (hip/vq.py): fp32 MFMA
distance + argmin, deterministic EMA statistics, straight-through gradient.
The M x K one-hot of the reference (vq.py:223, 233) is never materialised;
`embed_onehot` is therefore not kept (no caller reads it).
"""
from typing import Union

import torch
import torch.distributed as distributed
from torch import nn

from ..hip.vq import vq_codebook_pass, vq_train


def exists(val):
    return val is not None


def default(val, d):
    return val if exists(val) else d


def noop(*args, **kwargs):
    pass


def ema_inplace(moving_avg, new, decay):
    """vq.py:59-60 (host-side helper kept for API parity)."""
    moving_avg.data.mul_(decay).add_(new, alpha=(1 - decay))


def laplace_smoothing(x, n_categories, eps=1e-5):
    """vq.py:63-64 (host-side helper kept for API parity)."""
    return (x + eps) / (x.sum() + n_categories * eps)


class EuclideanCodebook(nn.Module):
    """vq.py:124-251 (kmeans_init=False, learnable_codebook=False on the hot path)."""

    def __init__(self, dim, codebook_size, kmeans_init=False, kmeans_iters=10, decay=0.8,
                 eps=1e-5, threshold_ema_dead_code=2, use_ddp=False, learnable_codebook=False,
                 sample_codebook_temp=0, emb_dropout=0.0):
        super().__init__()
        if kmeans_init or learnable_codebook or emb_dropout:
            raise NotImplementedError(
                "kmeans_init / learnable_codebook / emb_dropout are not on the TimeVQVAE path "
                "(configs never enable them)")
        self.decay = decay
        embed = torch.randn(codebook_size, dim)
        self.codebook_size = codebook_size
        self.kmeans_iters = kmeans_iters
        self.eps = eps
        self.threshold_ema_dead_code = threshold_ema_dead_code
        self.sample_codebook_temp = sample_codebook_temp
        self.emb_dropout = emb_dropout
        self.use_ddp = use_ddp
        self.all_reduce_fn = distributed.all_reduce if use_ddp else noop
        self.register_buffer("initted", torch.Tensor([not kmeans_init]))
        self.register_buffer("cluster_size", torch.zeros(codebook_size))
        self.register_buffer("embed_avg", embed.clone())
        self.learnable_codebook = learnable_codebook
        self.register_buffer("embed", embed)
        self.embed_onehot = None
        self.perplexity = None
        self.counts = None  # int32 (K,) per-code counts of the last pass (replaces embed_onehot)

    def _sync(self):
        if self.use_ddp and distributed.is_available() and distributed.is_initialized():
            return lambda t: distributed.all_reduce(t)
        return None

    @torch.no_grad()
    def forward(self, x, svq_temp: Union[float, None] = None):
        """Returns (quantize = E_old[idx], embed_ind); EMA update when training (vq.py:197-251).
        svq_temp > 0 samples idx ~ Categorical(softmax(dist / svq_temp)) (vq.py:216-222)."""
        if self.threshold_ema_dead_code > 0 and self.training:
            raise NotImplementedError("threshold_ema_dead_code > 0 is not on the TimeVQVAE path")
        shape = x.shape
        x3 = x.reshape(1, -1, shape[-1]) if x.dim() != 3 else x
        q, idx, _, perp, counts = vq_codebook_pass(
            x3, self.embed, self.cluster_size, self.embed_avg, straight_through=False,
            ema=self.training, decay=self.decay, eps=self.eps, sync=self._sync(),
            svq_temp=svq_temp)
        self.perplexity = perp
        self.counts = counts
        return q.reshape(shape), idx.reshape(shape[:-1])


_ZEROS = {}


def _eval_zero(device):
    key = torch.device(device)
    z = _ZEROS.get(key)
    if z is None:
        z = torch.zeros(1, device=key)
        if not (key.type == "cuda" and torch.cuda.is_current_stream_capturing()):
            _ZEROS[key] = z  # not from a graph's private pool (freed with the graph)
    return z


class VectorQuantize(nn.Module):
    """vq.py:255-407 (heads=1, codebook_dim=dim, channel_last, no orthogonal reg)."""

    def __init__(self, dim, codebook_size, codebook_dim=None, heads=1, decay=0.8, eps=1e-5,
                 kmeans_init=False, kmeans_iters=10, use_cosine_sim=False,
                 threshold_ema_dead_code=0, channel_last=True, accept_image_fmap=False,
                 commitment_weight=1.0, orthogonal_reg_weight=0.0,
                 orthogonal_reg_active_codes_only=False, orthogonal_reg_max_codes=None,
                 sample_codebook_temp=0.0, sync_codebook=False, emb_dropout=0.0, **kwargs):
        super().__init__()
        codebook_dim = default(codebook_dim, dim)
        if heads != 1 or codebook_dim != dim or use_cosine_sim or orthogonal_reg_weight > 0:
            raise NotImplementedError(
                "multi-head / projected / cosine / orthogonal-reg codebooks are not on the "
                "TimeVQVAE path (stage1.py:56-61 uses the defaults)")
        self.heads = heads
        self.project_in = nn.Identity()
        self.project_out = nn.Identity()
        self.eps = eps
        self.commitment_weight = commitment_weight
        self.orthogonal_reg_weight = orthogonal_reg_weight
        self._codebook = EuclideanCodebook(
            dim=codebook_dim, codebook_size=codebook_size, kmeans_init=kmeans_init,
            kmeans_iters=kmeans_iters, decay=decay, eps=eps,
            threshold_ema_dead_code=threshold_ema_dead_code, use_ddp=sync_codebook,
            learnable_codebook=False, sample_codebook_temp=sample_codebook_temp,
            emb_dropout=emb_dropout)
        self.codebook_size = codebook_size
        self.accept_image_fmap = accept_image_fmap
        self.channel_last = channel_last

    @property
    def codebook(self):
        return self._codebook.embed

    def forward(self, x, svq_temp: Union[float, None] = None):
        """x: (B,N,D) -> (quantize, embed_ind (B,N), vq_loss dict, perplexity)."""
        cb = self._codebook
        device = x.device
        vq_loss = {"loss": None, "commit_loss": 0.0, "orthogonal_reg_loss": 0.0}
        if self.accept_image_fmap:
            height, width = x.shape[-2:]
            x = x.flatten(2).transpose(1, 2)
        if not self.channel_last and not self.accept_image_fmap:
            x = x.transpose(1, 2)
        if self.training:
            if cb.threshold_ema_dead_code > 0:
                raise NotImplementedError("threshold_ema_dead_code > 0 is not on the path")
            quantize, embed_ind, commit, perp = vq_train(
                x, cb.embed, cb.cluster_size, cb.embed_avg, ema=True, decay=cb.decay, eps=cb.eps,
                sync=cb._sync(), svq_temp=svq_temp)
            if self.commitment_weight > 0:
                vq_loss["commit_loss"] = commit
                # vq.py:364's [0.] + commit * w, shape (1,): at w == 1 that is commit itself
                # (bit for bit), so no zeros / mul / add launches
                vq_loss["loss"] = (commit.reshape(1) if self.commitment_weight == 1.0
                                   else commit.reshape(1) * self.commitment_weight)
        else:
            with torch.no_grad():
                quantize, embed_ind, _, perp, counts = vq_codebook_pass(
                    x, cb.embed, cb.cluster_size, cb.embed_avg, straight_through=False,
                    ema=False, decay=cb.decay, eps=cb.eps, svq_temp=svq_temp)
            cb.counts = counts
        if vq_loss["loss"] is None:
            if self.training:
                vq_loss["loss"] = torch.zeros(1, device=device).requires_grad_(True)
            else:  # eval: a shared constant zero (no fill launch per call; never written)
                vq_loss["loss"] = _eval_zero(device)
        cb.perplexity = perp.detach() if perp is not None else None
        if not self.channel_last and not self.accept_image_fmap:
            quantize = quantize.transpose(1, 2)
        if self.accept_image_fmap:
            quantize = quantize.transpose(1, 2).reshape(quantize.shape[0], -1, height, width)
            embed_ind = embed_ind.reshape(embed_ind.shape[0], height, width)
        return quantize, embed_ind, vq_loss, cb.perplexity
