"""MaskGIT prior — same API as the reference timevqvae/models/bidirectional_transformer.py.

The reference builds its encoder from the third-party x-transformers package
(ContinuousTransformerWrapper + Encoder, bidirectional_transformer.py:92-110),
which is absent from this image.  `blocks` below restates that module tree with
the x-transformers 1.3x attribute names (project_in / post_emb_norm.gamma /
attn_layers.layers.{i}.{0.0.g | 1.to_q,to_k,to_v,to_out | 1.ff.0.0, 1.ff.2} /
attn_layers.final_norm.g / project_out) and its pre-norm semantics:

    x = project_in(x); x = post_emb_norm(x)             # LayerNorm, gamma only
    for (attn, ff) in depth: x = x + attn(RMSNorm(x)); x = x + ff(RMSNorm(x))
      (each branch skipped with prob layer_dropout in training)
    x = final RMSNorm(x); x = project_out(x)

attention: q,k,v,out bias-free Linear, head dim 64, softmax(QK^T/8) + dropout;
FF: Linear(+b) -> GELU -> Dropout -> Linear(+b).  PARITY UNPINNED: no reference
output exists for this part; project_in/out are bias-free
as in x-transformers >= 1.2x.
"""
import os
import random
from typing import Union

import torch
import torch.nn as nn

from ..hip import rng, streams
from ..hip.conv import PackCache, bn_eval_fusable, conv2d, conv2d_bn_eval
from ..hip.linear import gemm, linear, weight_product
from ..hip.norm import bn_snake
from ..hip.xf import (attn_branch, attn_branch_supported, batch_colsum, drop_first_token,
                      embed_assemble, embedding, fused_ff, fused_ff_supported, gelu,
                      layer_norm, linear_act, prior_lf_eval, prior_lf_eval_sample,
                      prior_lf_eval_supported, prior_lf_eval_workspace, qkv_attention, rmsnorm, rmsnorm_res,
                      upsample_nearest_t)
from ..hip._native import call, grad_sink, ptr, stream_ptr, value
from ..hip.sample import codebook_gather_nchw, full_tokens, maskgit_sample, tied_logits_sample
from ..hip.upscale import supported as ups_supported
from ..hip.upscale import (hf_embed_folded, hf_embed_supported, upsample_conv_gelu,
                           upsample_conv_gelu_bn_eval)

# the HF prior's sampling step straight from its head (no logits in memory); 0: form the
# logits and sample them (A/B and diagnosis)
FUSED_SAMPLE = True
# Upscale's first conv on the LF token grid (hip.upscale); False: upsample, then conv (tests)
UPS_ON_TOKENS = True
HEAD_FOLD = True  # False (tests): project_out and pred_head's Linear as two GEMMs
HF_EMBED_FOLD = True  # False (tests): Upscale's last conv and project_in unfolded


# ------------------------------------------------------------------ x-transformers tree
class RMSNorm(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.scale = dim ** 0.5
        self.g = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        return rmsnorm(x, self.g)


class LayerNorm(nn.Module):
    """x-transformers LayerNorm: F.layer_norm without affine, times gamma."""

    def __init__(self, dim):
        super().__init__()
        self.gamma = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        return layer_norm(x, self.gamma, None, 1e-5)


class Attention(nn.Module):
    def __init__(self, dim, heads, dim_head=64, dropout=0.0):
        super().__init__()
        inner = heads * dim_head
        self.heads = heads
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_k = nn.Linear(dim, inner, bias=False)
        self.to_v = nn.Linear(dim, inner, bias=False)
        self.to_out = nn.Linear(inner, dim, bias=False)
        self.dropout = dropout
        self._site = rng.new_site()

    def forward(self, x, residual, gate=None):
        o = qkv_attention(x, self.to_q.weight, self.to_k.weight, self.to_v.weight, self.heads,
                          self.dropout if self.training else 0.0, self._site)
        return linear(o, self.to_out.weight, None, residual=residual, gate=gate)


class FeedForward(nn.Module):
    def __init__(self, dim, mult=1, dropout=0.0):
        super().__init__()
        inner = int(dim * mult)
        self.ff = nn.Sequential(nn.Sequential(nn.Linear(dim, inner), nn.GELU()), nn.Dropout(dropout),
                                nn.Linear(inner, dim))
        self._site = rng.new_site()

    def forward(self, x, residual, gate=None):
        lin1 = self.ff[0][0]
        p = self.ff[1].p if self.training else 0.0
        lin2 = self.ff[2]
        if fused_ff_supported(x, lin1.weight, lin2.weight):
            # the whole branch + residual in one launch each way (hip.xf.fused_ff)
            return fused_ff(x, residual, lin1.weight, lin1.bias, lin2.weight, lin2.bias, gate, p,
                            self._site)
        h = linear_act(x, lin1.weight, lin1.bias, gelu=True)
        if p > 0:
            h = dropout(h, p, self._site)
        lin2 = self.ff[2]
        return linear(h, lin2.weight, lin2.bias, residual=residual, gate=gate)


class Residual(nn.Module):
    def forward(self, x, residual):
        return x + residual


class Encoder(nn.Module):
    """x-transformers Encoder(pre_norm=True, ...) restated.

    Layer dropout: in training each branch is skipped with probability layer_dropout
    (x-transformers draws `random() < layer_dropout` per branch).  `_touched[i]` records
    whether branch i ran in any forward since the optimizer's last zero_grad; its
    parameters carry `_tvq_gate = (self, i)`, so FusedAdamW leaves a skipped branch's
    parameters untouched, as torch.optim.AdamW does for parameters whose .grad is None."""

    def __init__(self, dim, depth, heads, attn_dim_head=64, use_rmsnorm=True, ff_mult=1,
                 layer_dropout=0.0, attn_dropout=0.0, ff_dropout=0.0):
        super().__init__()
        self.dim = dim
        norm = (lambda: RMSNorm(dim)) if use_rmsnorm else (lambda: LayerNorm(dim))
        self.layers = nn.ModuleList()
        self.layer_types = ("a", "f") * depth
        for t in self.layer_types:
            block = (Attention(dim, heads, attn_dim_head, attn_dropout) if t == "a"
                     else FeedForward(dim, ff_mult, ff_dropout))
            self.layers.append(nn.ModuleList([nn.ModuleList([norm(), None, None]), block, Residual()]))
        self.layer_dropout = layer_dropout
        self.final_norm = norm()
        n = len(self.layers)
        self.register_buffer("_keep", torch.ones(n), persistent=False)
        self.register_buffer("_touched", torch.ones(n), persistent=False)
        for i, layer in enumerate(self.layers):
            for p in layer.parameters():
                p._tvq_gate = (self, i)
        self._site = rng.new_site()
        self._epoch = -1
        self._touched_host = [1.0] * n

    def _draw_branches(self, device):
        """Per-branch keep decisions of this forward; updates `_touched`.  Returns the
        host keep list (eager) or None (device decisions: `_keep` holds them)."""
        from ..hip.optim import grad_epoch
        fresh = self._epoch != grad_epoch()
        self._epoch = grad_epoch()
        n = len(self.layers)
        if rng.decisions_on_device():
            # graph capture: the decisions are re-drawn on every replay
            call("tvq_layer_drop", ptr(rng.seed_tensor(device)), rng.call_offset(self._site),
                 float(self.layer_dropout), n, ptr(self._keep), ptr(self._touched),
                 int(not fresh), stream_ptr())
            return None
        keep = [0.0 if random.random() < self.layer_dropout else 1.0 for _ in range(n)]
        self._touched_host = keep if fresh else [max(a, b) for a, b in zip(self._touched_host, keep)]
        self._touched.copy_(torch.tensor(self._touched_host))
        return keep

    def forward(self, x):
        keep = None
        device_gates = False
        if self.training and self.layer_dropout > 0.0:
            keep = self._draw_branches(x.device)
            device_gates = keep is None
        elif self.training and self._touched_host != [1.0] * len(self.layers):
            self._touched_host = [1.0] * len(self.layers)
            self._touched.fill_(1.0)
        for i, (norms, block, _) in enumerate(self.layers):
            if keep is not None and keep[i] == 0.0:
                continue
            # device gates (graph capture): x + keep_i * branch, the gate applied in the
            # branch's output-Linear epilogue (its backward scales the branch gradient)
            gate = self._keep[i:i + 1] if device_gates else None
            if isinstance(norms[0], RMSNorm):
                if isinstance(block, Attention) and attn_branch_supported(x, norms[0].g, block):
                    # RMSNorm + attention + out-projection + gated residual: one launch each way
                    x = attn_branch(x, norms[0].g, block, gate,
                                    block.dropout if self.training else 0.0)
                    continue
                n, r = rmsnorm_res(x, norms[0].g)  # residual gradient summed in the norm bwd
                x = block(n, residual=r, gate=gate)
            else:
                x = block(norms[0](x), residual=x, gate=gate)
        return self.final_norm(x)


class ContinuousTransformerWrapper(nn.Module):
    def __init__(self, dim_in, dim_out, max_seq_len, attn_layers, use_abs_pos_emb=False,
                 post_emb_norm=True):
        super().__init__()
        if use_abs_pos_emb:
            raise NotImplementedError("abs pos emb is off on the path (use_abs_pos_emb=False)")
        dim = attn_layers.dim
        self.max_seq_len = max_seq_len
        self.post_emb_norm = LayerNorm(dim) if post_emb_norm else nn.Identity()
        self.attn_layers = attn_layers
        self.project_in = nn.Linear(dim_in, dim, bias=False)
        self.project_out = nn.Linear(dim, dim_out, bias=False)

    def forward(self, x):
        return self.forward_projected(linear(x, self.project_in.weight))

    def forward_projected(self, x, project_out=True):
        """forward() after project_in (its input already projected, e.g. by the HF prior's
        folded embedding); project_out=False: without project_out (folded into the head)."""
        x = self.post_emb_norm(x)
        if not project_out:
            return self.attn_layers(x)
        x = self.attn_layers(x)
        return linear(x, self.project_out.weight)


# ------------------------------------------------------------------ helper ops
class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, site):
        x = x.contiguous()
        y = torch.empty_like(x)
        seed = rng.seed_tensor(x.device)
        off = rng.call_offset(site)
        call("tvq_dropout_bwd", ptr(x), x.numel(), float(p), ptr(seed), off, ptr(y), stream_ptr())
        ctx.cfg = (p, off)
        ctx.seed = seed
        return y

    @staticmethod
    def backward(ctx, g):
        p, off = ctx.cfg
        g = g.contiguous()
        dx = torch.empty_like(g)
        call("tvq_dropout_bwd", ptr(g), g.numel(), float(p), ptr(ctx.seed), off, ptr(dx), stream_ptr())
        return dx, None, None


def dropout(x, p, site):
    return _Dropout.apply(x, float(p), int(site))


class _TiedLogits(torch.autograd.Function):
    """logits = embed @ W[:K]^T + bias[:, :K]  (bidirectional_transformer.py:186-191; the
    mask-token column K is never computed since it is dropped)."""

    @staticmethod
    def forward(ctx, h, W, bias, K):
        B, n, D = h.shape
        h2 = h.reshape(B * n, D).contiguous()
        M = B * n
        out = gemm(h2, D, 1, W, 1, D, M, K, D, R=bias, ldr=bias.shape[1], rmod=n)
        ctx.save_for_backward(h2, W)
        ctx.W, ctx.bias = W, bias
        ctx.cfg = (B, n, D, K, tuple(bias.shape))
        return out.reshape(B, n, K)

    @staticmethod
    def backward(ctx, g):
        h2, W = ctx.saved_tensors
        B, n, D, K, bshape = ctx.cfg
        M = B * n
        g2 = g.reshape(M, K).contiguous()
        dh = dW = dbias = None
        if ctx.needs_input_grad[0]:
            dh = gemm(g2, K, 1, W, D, 1, M, D, K).reshape(B, n, D)
        if ctx.needs_input_grad[1]:
            sink = grad_sink(ctx.W)
            if sink is not None:  # tied table: accumulate next to the embedding-lookup grad
                # (both on the aux stream of this stream, so their order is fixed)
                with streams.offload(g2, h2):
                    gemm(g2, 1, K, h2, D, 1, K, D, M, out=sink, ldc=D, accumulate=True)
            else:
                dW = torch.zeros_like(W)
                gemm(g2, 1, K, h2, D, 1, K, D, M, out=dW, ldc=D)
        if ctx.needs_input_grad[2]:
            # sum over the batch into the (n, K+1) table's first K columns, in order
            sink = grad_sink(ctx.bias)
            if sink is not None:
                with streams.offload(g2):
                    batch_colsum(g2.reshape(B, n, K), sink, bshape[1], True)
            else:
                dbias = torch.zeros(bshape, device=g.device)
                batch_colsum(g2.reshape(B, n, K), dbias, bshape[1], False)
        return dh, dW, dbias, None


TIED_CE_FUSED = True  # False (tests): logits GEMM + masked CE forward / backward launches


def tied_ce_supported(h, W, K):
    """Fused for both priors: at the LF prior's 6144 tokens the kernel is slower alone (96
    blocks, ~100 us against ~70 us for the unfused launches) but the joint step is 0.02 ms
    faster with it (fewer launches and no logits round trip; tools/step_ab.py, same box:
    3.915-3.928 vs 3.940-3.947 ms)."""
    return (h.is_cuda and h.dim() == 3 and h.shape[-1] == 128 and W.shape[1] == 128
            and K in (64, 128, 256, 512) and W.shape[0] >= K)


class _TiedLogitsCE(torch.autograd.Function):
    """masked_cross_entropy(h @ W[:K]^T + bias[:, :K], target, keep) for a backward that starts
    at this loss with root gradient `gscale` (MaskGIT.forward_backward): tvq_tied_logits_ce
    computes the loss, the logits' gradient D and dh = D W[:K] in the forward, the logits never
    reaching memory (bidirectional_transformer.py:186-191, maskgit.py:183-191).  The backward
    adds the tied-table and bias gradients (D^T h, the batch column sums of D) and returns dh;
    a root gradient other than `gscale` (not the forward_backward use) rescales them first."""

    @staticmethod
    def forward(ctx, h, W, bias, K, target, keep, gscale):
        B, n, D = h.shape
        M = B * n
        h2 = h.reshape(M, D).contiguous()
        dev = h.device
        ws = torch.empty(value("tvq_tied_logits_ce_workspace", M, K), device=dev)
        dl = torch.empty((M, K), device=dev)
        dh = torch.empty((M, D), device=dev)
        out = torch.empty(2, device=dev)
        call("tvq_tied_logits_ce", ptr(h2), M, D, ptr(W.contiguous()), K, ptr(bias), bias.shape[0],
             bias.stride(0), ptr(target.reshape(-1).contiguous()),
             ptr(keep.reshape(-1).contiguous()), ptr(gscale), ptr(dl), ptr(dh), ptr(out), ptr(ws),
             stream_ptr())
        ctx.save_for_backward(h2, dl, dh, gscale)
        ctx.W, ctx.bias = W, bias
        ctx.cfg = (B, n, D, K, tuple(bias.shape))
        return out[0]

    @staticmethod
    def backward(ctx, g):
        h2, dl, dh, gscale = ctx.saved_tensors
        B, n, D, K, bshape = ctx.cfg
        M = B * n
        if g.data_ptr() != gscale.data_ptr():  # another root gradient: D, dh scale by g / gscale
            from ..hip.linear import scale_by
            r = torch.empty(1, device=g.device)
            call("tvq_scalar_ratio", ptr(g.reshape(1).contiguous()), ptr(gscale), ptr(r), stream_ptr())
            dl, dh = scale_by(dl, r), scale_by(dh, r)
        need = ctx.needs_input_grad
        dW = dbias = None
        if need[1]:
            sink = grad_sink(ctx.W)
            if sink is not None:
                with streams.offload(dl, h2):
                    gemm(dl, 1, K, h2, D, 1, K, D, M, out=sink, ldc=D, accumulate=True)
            else:
                dW = torch.zeros_like(ctx.W)
                gemm(dl, 1, K, h2, D, 1, K, D, M, out=dW, ldc=D)
        if need[2]:
            sink = grad_sink(ctx.bias)
            if sink is not None:
                with streams.offload(dl):
                    batch_colsum(dl.view(B, n, K), sink, bshape[1], True)
            else:
                dbias = torch.zeros(bshape, device=g.device)
                batch_colsum(dl.view(B, n, K), dbias, bshape[1], False)
        return (dh.view(B, n, D) if need[0] else None), dW, dbias, None, None, None, None


def tied_logits_ce(h, W, bias, K, target, keep, gscale):
    """The prior's masked CE loss from its head output h (B, n, 128) in one fused pass; the
    backward is meant to start here with root gradient `gscale` (see _TiedLogitsCE)."""
    return _TiedLogitsCE.apply(h, W, bias, int(K), target, keep, gscale)


class Upscale(nn.Module):
    """bidirectional_transformer.py:12-30: nearest x(m/n) -> Conv1d(k3) -> GELU -> BN1d -> Conv1d(k3)."""

    def __init__(self, in_channels: int, out_channels: int, h_dim: int) -> None:
        super().__init__()
        self.conv = nn.Sequential(
            nn.Conv1d(in_channels, h_dim, kernel_size=3, stride=1, padding=1),
            nn.GELU(),
            nn.BatchNorm1d(h_dim),
            nn.Conv1d(h_dim, out_channels, kernel_size=3, stride=1, padding=1),
        )

    def forward(self, x, upscale_size: int):
        """x: (b n d) -> (b m d)."""
        x = self.first(x, upscale_size)
        c = self.conv
        x = conv2d(x, c[3].weight, c[3].bias)
        return x.transpose(1, 2)                         # b m d

    def first(self, x, upscale_size: int):
        """BN(GELU(conv(interpolate(x^T, m)))) -> (b, H, m).  For an integer ratio m / n >= 2
        the conv runs on the n tokens (hip.upscale: f x fewer FLOPs, the upsampled input is
        never formed); otherwise upsample then conv."""
        c = self.conv
        w, b, bn = c[0].weight, c[0].bias, c[2]
        if UPS_ON_TOKENS and ups_supported(x, upscale_size, w):
            if bn_eval_fusable(x, bn, w, b):  # sampling: GEMM + one combine launch
                return upsample_conv_gelu_bn_eval(x, upscale_size, w, b, bn)
            return bn_snake(upsample_conv_gelu(x, upscale_size, w, b), bn, None)
        x = upsample_nearest_t(x, upscale_size)          # b n d -> b d m, one kernel
        if bn_eval_fusable(x, bn, w, b):  # eval: one launch
            return conv2d_bn_eval(x, w, b, bn, None, pre_gelu=True)
        return bn_snake(gelu(conv2d(x, w, b)), bn, None)


# ------------------------------------------------------------------ the prior
class BidirectionalTransformer(nn.Module):
    def __init__(self, kind: str, num_tokens: int, codebook_sizes: dict, embed_dim: int,
                 hidden_dim: int, n_layers: int, heads: int, ff_mult: int, use_rmsnorm: bool,
                 p_unconditional: float, n_classes: int, model_dropout: float = 0.3,
                 emb_dropout: float = 0.3, **kwargs):
        super().__init__()
        kind = kind.lower()
        assert kind in ["lf", "hf"], "invalid `kind`."
        self.kind = kind
        self._eval_ws = {}  # (device, n) -> packed-weight workspace of the LF eval launch
        self.num_tokens = num_tokens
        self.n_classes = n_classes
        self.p_unconditional = p_unconditional
        in_dim = embed_dim if kind == "lf" else 2 * embed_dim
        out_dim = embed_dim
        self.emb_dropout = emb_dropout
        self.mask_token_ind = {"lf": codebook_sizes["lf"], "hf": codebook_sizes["hf"]}
        self.tok_emb_l = nn.Embedding(codebook_sizes["lf"] + 1, embed_dim)
        if kind == "hf":
            self.tok_emb_h = nn.Embedding(codebook_sizes["hf"] + 1, embed_dim)
        self.pos_emb = nn.Embedding(self.num_tokens + 1, in_dim)
        self.class_condition_emb = nn.Embedding(n_classes + 1, in_dim)
        self.blocks = ContinuousTransformerWrapper(
            dim_in=in_dim, dim_out=in_dim, max_seq_len=self.num_tokens + 1, use_abs_pos_emb=False,
            post_emb_norm=True,
            attn_layers=Encoder(dim=hidden_dim, depth=n_layers, heads=heads, attn_dim_head=64,
                                use_rmsnorm=use_rmsnorm, ff_mult=ff_mult,
                                layer_dropout=model_dropout, attn_dropout=model_dropout,
                                ff_dropout=model_dropout))
        self.pred_head = nn.Sequential(nn.Linear(in_features=in_dim, out_features=out_dim),
                                       nn.GELU(), nn.LayerNorm(out_dim, eps=1e-12))
        codebook_size = codebook_sizes["lf"] if kind == "lf" else codebook_sizes["hf"]
        self.codebook_size = codebook_size
        self.bias = nn.Parameter(torch.zeros(self.num_tokens, codebook_size + 1))
        if kind == "hf":
            self.projector = Upscale(embed_dim, embed_dim, 2 * embed_dim)
        self._site_l = rng.new_site()
        self._site_h = rng.new_site()
        self._class_rand = None

    def class_embedding(self, class_condition: Union[None, torch.Tensor], batch_size: int, device):
        """bidirectional_transformer.py:124-150.  `_class_rand` (tests only): the uniform
        draws of the classifier-free-guidance drop, injected instead of torch.rand."""
        if class_condition is None:
            idx = full_tokens((batch_size, 1), self.n_classes, device)
        elif self.training:
            # drop to the null class where u > p fails, u ~ U[0,1) per sample: one kernel
            # (the device counter RNG; the reference's torch.rand draws can be injected)
            y = class_condition.long().reshape(-1).contiguous()
            idx = torch.empty_like(y)
            u = self._class_rand
            rnd = (torch.as_tensor(u).to(device=device, dtype=torch.float32).reshape(-1).contiguous()
                   if u is not None else None)
            seed = rng.seed_tensor(device) if rnd is None else None
            off = rng.call_offset(self._site_l) if rnd is None else 0
            call("tvq_class_index", ptr(y), y.numel(), float(self.p_unconditional), self.n_classes,
                 ptr(seed), off, ptr(rnd), ptr(idx), stream_ptr())
            idx = idx.reshape(class_condition.shape)
        else:
            idx = class_condition.long()
        return embedding(idx, self.class_condition_emb.weight)  # (b 1 dim)

    def _tok(self, s, table, kind, site):
        p = self.emb_dropout if self.training else 0.0
        return embedding(s, table, self.mask_token_ind[kind], p, site)

    def _head(self, x):
        lin, ln = self.pred_head[0], self.pred_head[2]
        h = linear_act(x, lin.weight, lin.bias, gelu=True)
        return layer_norm(h, ln.weight, ln.bias, ln.eps)

    def _blocks_head(self, x, projected=False):
        """pred_head(drop_first(blocks(x))) (bidirectional_transformer.py:186-191,233-236).
        HEAD_FOLD: project_out and pred_head's Linear meet without a nonlinearity, so they run
        as one Linear with W_p W_out (hip.linear.weight_product): the (B, n + 1, in_dim)
        project_out output is never formed (the same function up to fp32 reassociation).
        projected: x has already been through project_in."""
        blk = self.blocks
        if not HEAD_FOLD:
            x = blk.forward_projected(x) if projected else blk(x)
            return self._head(drop_first_token(x))
        if not projected:
            x = linear(x, blk.project_in.weight)
        x = drop_first_token(blk.forward_projected(x, project_out=False))
        lin, ln = self.pred_head[0], self.pred_head[2]
        h = linear_act(x, weight_product(lin.weight, blk.project_out.weight), lin.bias, gelu=True)
        return layer_norm(h, ln.weight, ln.bias, ln.eps)

    def forward_lf(self, s_M_l, class_condition: Union[None, torch.Tensor] = None):
        """bidirectional_transformer.py:166-192."""
        if prior_lf_eval_supported(self, s_M_l):
            # eval (sampling): the whole prior as one launch per step (hip.xf.prior_lf_eval)
            return prior_lf_eval(self, s_M_l, class_condition)
        return _TiedLogits.apply(self._embed_lf(s_M_l, class_condition), self.tok_emb_l.weight,
                                 self.bias, self.codebook_size)

    def _embed_lf(self, s_M_l, class_condition):
        device = s_M_l.device
        tok = self._tok(s_M_l, self.tok_emb_l.weight, "lf", self._site_l)
        cls_emb = self.class_embedding(class_condition, s_M_l.shape[0], device)
        n = tok.shape[1]
        embed = embed_assemble(cls_emb, tok, None, self.pos_emb.weight, n)  # cat(cls, tok + pos)
        return self._blocks_head(embed)

    def forward_hf(self, s_M_l, s_M_h, class_condition=None):
        """bidirectional_transformer.py:194-236."""
        return _TiedLogits.apply(self._embed_hf(s_M_l, s_M_h, class_condition),
                                 self.tok_emb_h.weight, self.bias, self.codebook_size)

    def _embed_hf(self, s_M_l, s_M_h, class_condition):
        device = s_M_l.device
        tl = self._tok(s_M_l, self.tok_emb_l.weight, "lf", self._site_l)
        th = self._tok(s_M_h, self.tok_emb_h.weight, "hf", self._site_h)
        n = th.shape[1]
        if HF_EMBED_FOLD:
            x = self.projector.first(tl, n)  # (b, H, m)
            W_in = self.blocks.project_in.weight
            up = self.projector.conv
            if hf_embed_supported(x, th, W_in, up[3].weight, self.pos_emb.weight):
                # Upscale's last conv and project_in as one folded op (hip.upscale)
                cls_emb = self.class_embedding(class_condition, s_M_l.shape[0], device)
                z = hf_embed_folded(x, th, cls_emb, W_in, up[3].weight, up[3].bias,
                                    self.pos_emb.weight)
                return self._blocks_head(z, projected=True)
            tl = conv2d(x, up[3].weight, up[3].bias).transpose(1, 2)
        else:
            tl = self.projector(tl, upscale_size=n)
        cls_emb = self.class_embedding(class_condition, s_M_l.shape[0], device)
        # cat(cls, cat(tl, th, -1) + pos) in one kernel
        embed = embed_assemble(cls_emb, tl, th, self.pos_emb.weight, n)
        return self._blocks_head(embed)

    def sample(self, s_M_l, s_M_h=None, class_condition=None, mask_id=None, gumbel=None,
               site=0, want_logits=False, first=True):
        """One categorical draw per token of this prior's logits (maskgit.py:302-326): the
        sampled codes (known tokens -- the ones != mask_id of the band being decoded -- kept)
        and p(sampled) (+inf for known tokens).  The HF prior in eval mode draws straight
        from its head (hip.sample.tied_logits_sample: the logits never reach memory);
        otherwise the logits are formed and hip.sample.maskgit_sample draws from them.
        want_logits: also return the logits (tests).  first=False: the weights are those of
        the previous call (the decoding steps after a pass's first), so the LF launch reuses
        their packed copy."""
        s = s_M_l if self.kind == "lf" else s_M_h
        if self.kind == "lf" and FUSED_SAMPLE and prior_lf_eval_supported(self, s_M_l):
            key = (s_M_l.device, s_M_l.shape[1])
            ws = self._eval_ws.get(key)
            fresh = ws is None
            if fresh:
                ws = prior_lf_eval_workspace(self, s_M_l)
                self._eval_ws[key] = ws
            return prior_lf_eval_sample(self, s_M_l, class_condition, mask_id, gumbel=gumbel,
                                        site=site, want_logits=want_logits, ws=ws,
                                        ready=not (first or fresh))
        if (self.kind == "hf" and not self.training and FUSED_SAMPLE
                and self.tok_emb_h.weight.shape[1] in (64, 128)):
            return tied_logits_sample(self._head_hf_eval(s_M_l, s_M_h, class_condition),
                                      self.tok_emb_h.weight, self.bias, self.codebook_size, s,
                                      mask_id, gumbel=gumbel, site=site, want_logits=want_logits)
        logits = self(s_M_l, s_M_h, class_condition) if self.kind == "hf" else \
            self(s_M_l, class_condition=class_condition)
        out = maskgit_sample(logits, s, mask_id, gumbel=gumbel, site=site)
        return out + (logits,) if want_logits else out

    @torch.no_grad()
    def _head_hf_eval(self, s_M_l, s_M_h, class_condition):
        """The HF prior's head output in eval mode (the input of the tied logits), with the
        Linears that meet without a nonlinearity between them composed (weights fixed while
        sampling; the same function up to fp32 reassociation):
          * project_in after cat(Upscale(tl), th) + pos: its tl half folds into Upscale's
            last conv (256 -> 32 output channels instead of 256 -> 128 then 128 -> 32), its
            th half into the token table (tok_emb_h W_in[:, D:]^T, gathered per token), and
            the position / class tables are projected once;
          * project_out then pred_head's Linear: one 32 -> 128 Linear (W_p W_out).
        The (B, n + 1, 2 D) embedding and the (B, n, 2 D) project_out output are never
        formed.  bidirectional_transformer.py:12-30, 194-236."""
        from ..hip.linear import gemm
        dev = s_M_l.device
        B, n = s_M_h.shape
        D = self.tok_emb_h.weight.shape[1]
        W_in = self.blocks.project_in.weight  # (d, 2 D)
        d = W_in.shape[0]
        up = self.projector.conv
        W2, b2 = up[3].weight, up[3].bias  # (D, H, 3), (D)
        H = W2.shape[1]
        # folded tables / weights (tiny GEMMs)
        W2c = gemm(W_in, 2 * D, 1, W2, H * 3, 1, d, H * 3, D).view(d, H, 3)
        b2c = gemm(W_in, 2 * D, 1, b2, 1, 1, d, 1, D).view(d)
        Th = gemm(self.tok_emb_h.weight, D, 1, W_in[:, D:], 1, 2 * D,
                  self.tok_emb_h.weight.shape[0], d, D)
        P = gemm(self.pos_emb.weight, 2 * D, 1, W_in, 1, 2 * D, self.pos_emb.weight.shape[0], d,
                 2 * D)
        C = gemm(self.class_condition_emb.weight, 2 * D, 1, W_in, 1, 2 * D,
                 self.class_condition_emb.weight.shape[0], d, 2 * D)
        lin, ln = self.pred_head[0], self.pred_head[2]
        W_out = self.blocks.project_out.weight  # (2 D, d)
        Wc = gemm(lin.weight, 2 * D, 1, W_out, d, 1, lin.weight.shape[0], d, 2 * D)
        # x1 = cat(C[cls], Upscale'(tl) + Th[s_h] + P[:n]) = project_in(embed)
        tl = self._tok(s_M_l, self.tok_emb_l.weight, "lf", self._site_l)
        x = self.projector.first(tl, n)
        r = codebook_gather_nchw(s_M_h, Th, 1, n).view(B, d, n)  # Th[s_h] channels-first
        with PackCache.paused():  # W2c is computed per call: never cached
            u = conv2d(x, W2c, b2c, residual=r)  # (B, d, n)
        if class_condition is None:
            idx = full_tokens((B, 1), self.n_classes, dev)
        else:
            idx = class_condition.long()
        x = embed_assemble(embedding(idx, C), u.transpose(1, 2), None, P, n)
        x = self.blocks.post_emb_norm(x)
        x = self.blocks.attn_layers(x)
        h = linear_act(drop_first_token(x), Wc, lin.bias, gelu=True)
        return layer_norm(h, ln.weight, ln.bias, ln.eps)

    def forward(self, s_M_l, s_M_h=None, class_condition: Union[None, torch.Tensor] = None):
        if self.kind == "lf":
            return self.forward_lf(s_M_l, class_condition)
        return self.forward_hf(s_M_l, s_M_h, class_condition)
