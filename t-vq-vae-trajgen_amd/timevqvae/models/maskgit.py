"""MaskGIT (stage2) — same API as the reference timevqvae/models/maskgit.py.

Training forward (maskgit.py:155-192): frozen stage1 encoders in eval mode (one
fused STFT pass for both branches, eval BN+Snake, VQ assign), on-device random
masking (_randomly_mask_tokens, no host loop), the two bidirectional
transformers, and a fused masked cross-entropy.  Iterative decoding
(maskgit.py:294-446) runs one fused HIP sampling kernel per step with no host
synchronisation (the reference's per-row Python loop and .item() are gone).
"""
import os
from typing import Callable, Union

import numpy as np
import torch
import torch.nn as nn

from ..hip import rng, streams, wgrad
from ..hip.sample import (codebook_gather_nchw, full_tokens, mask_len, maskgit_remask,
                          maskgit_sample)
from ..hip.signal import stft_encode
from ..hip.loss import add_losses
from ..hip.vq import indices_only
from ..hip.xf import mask_tokens, masked_cross_entropy
from ..utils import freeze, quantize, zero_pad_high_freq, zero_pad_low_freq
from . import bidirectional_transformer as bt
from .bidirectional_transformer import BidirectionalTransformer
from .vq import VectorQuantize
from .vq_vae import VQVAEEncoder


def _latent_width(T: int, n_enc_blocks: int) -> int:
    W = T + 1
    for _ in range(n_enc_blocks):
        W = (W + 2 - 4) // 2 + 1
    return W




class MaskGIT(nn.Module):
    """ref: maskgit.py:20-477 (ESS / self-token-critic paths are disabled by config)."""

    def __init__(self, stage1_ckpt_fname: str, input_length: int, in_channels: int, config: dict,
                 n_classes: int, choice_temperatures: dict, T: dict, **kwargs):
        super().__init__()
        self.choice_temperature_l = choice_temperatures["lf"]
        self.choice_temperature_h = choice_temperatures["hf"]
        self.T = T
        self.config = config
        self.n_classes = n_classes
        self.n_fft = config["VQ-VAE"]["n_fft"]
        self.cfg_scale = config["MaskGIT"]["cfg_scale"]
        self.mask_token_ids = {"lf": config["VQ-VAE"]["codebook_sizes"]["lf"],
                               "hf": config["VQ-VAE"]["codebook_sizes"]["hf"]}
        self.gamma = self.gamma_func("cosine")
        from ..trainers.stage1 import Stage1  # circular import, as in the reference
        stage1 = kwargs.get("stage1")
        if stage1 is None and stage1_ckpt_fname is None:
            # weights to follow (Stage2.load_from_checkpoint: stage2.ckpt holds stage1's)
            stage1 = Stage1(input_length, in_channels, config)
        elif stage1 is None:
            stage1 = Stage1.load_from_checkpoint(stage1_ckpt_fname, input_length=input_length,
                                                 in_channels=in_channels, config=config,
                                                 map_location="cpu")
        self.stage1 = stage1
        freeze(self.stage1)
        self.stage1.eval()
        self.encoder_l = self.stage1.encoder_l
        self.decoder_l = self.stage1.decoder_l
        self.vq_model_l = self.stage1.vq_model_l
        self.encoder_h = self.stage1.encoder_h
        self.decoder_h = self.stage1.decoder_h
        self.vq_model_h = self.stage1.vq_model_h
        for enc in (self.encoder_l, self.encoder_h):
            if int(enc.num_tokens) == 0:  # never run: derive H', W' from the conv plan
                n_enc = sum(1 for m in enc.encoder if type(m).__name__ == "VQVAEEncBlock")
                enc.H_prime = torch.tensor(3)
                enc.W_prime = torch.tensor(_latent_width(input_length, n_enc))
                enc.num_tokens = enc.H_prime * enc.W_prime
        self.num_tokens_l = int(self.encoder_l.num_tokens)
        self.num_tokens_h = int(self.encoder_h.num_tokens)
        self.H_prime_l, self.H_prime_h = int(self.encoder_l.H_prime), int(self.encoder_h.H_prime)
        self.W_prime_l, self.W_prime_h = int(self.encoder_l.W_prime), int(self.encoder_h.W_prime)
        emb_dim = self.config["encoder"]["hid_dim"]
        self.transformer_l = BidirectionalTransformer(
            "lf", self.num_tokens_l, config["VQ-VAE"]["codebook_sizes"], emb_dim,
            **config["MaskGIT"]["prior_model_l"], n_classes=n_classes)
        self.transformer_h = BidirectionalTransformer(
            "hf", self.num_tokens_h, config["VQ-VAE"]["codebook_sizes"], emb_dim,
            **config["MaskGIT"]["prior_model_h"], n_classes=n_classes,
            num_tokens_l=self.num_tokens_l)
        self._site_mask_l = rng.new_site()
        self._site_mask_h = rng.new_site()
        self._site_sample = rng.new_site()

    def train(self, mode: bool = True):
        super().train(mode)
        self.stage1.eval()  # stage1 stays frozen in eval mode (maskgit.py:61-62,161-164)
        return self

    @torch.no_grad()
    def encode_to_z_q(self, x, encoder: VQVAEEncoder, vq_model: VectorQuantize,
                      svq_temp: Union[float, None] = None):
        """maskgit.py:117-134."""
        z = encoder(x)
        zq, s, _, _ = quantize(z, vq_model, svq_temp=svq_temp)
        return zq, s

    @torch.no_grad()
    def encode_tokens(self, x):
        """Both branches from one fused STFT pass: (s_l (b n), s_h (b m)) int64."""
        st = stft_encode(x, enc_l=True, enc_h=True)
        with indices_only():  # the tokens only: no per-code counts / perplexity launches
            with streams.branch(x.device) as br:  # HF encoder concurrently with LF
                br.inputs(st)
                _, s_h, _, _ = quantize(self.encoder_h.encode_timefreq(st["enc_h"]), self.vq_model_h)
                br.outputs(s_h)
            _, s_l, _, _ = quantize(self.encoder_l.encode_timefreq(st["enc_l"]), self.vq_model_l)
        br.join()
        return s_l, s_h

    def masked_prediction(self, transformer, class_condition, *s_in):
        """maskgit.py:136-153 (classifier-free guidance)."""
        if class_condition is None:
            return transformer(*s_in, class_condition=None)
        if self.cfg_scale == 1.0:
            return transformer(*s_in, class_condition=class_condition)
        logits_null = transformer(*s_in, class_condition=None)
        logits = transformer(*s_in, class_condition=class_condition)
        return logits_null + self.cfg_scale * (logits - logits_null)

    def forward(self, x, y, draws=None):
        """maskgit.py:155-192 -> (loss, (loss_l, loss_h)).

        `draws` (tests only) injects the reference's random draws instead of the device
        RNG: {"ratio_l", "rand_l", "ratio_h", "rand_h"} for _randomly_mask_tokens
        (np.random.uniform ratios, torch.rand scores) and {"cls_l", "cls_h"} for the
        class-drop draws of each transformer (bidirectional_transformer.py:140-143)."""
        loss_l, loss_h = self._priors(x, y, draws, None)
        return add_losses(loss_l, loss_h), (loss_l, loss_h)

    def forward_backward(self, x, y, one, draws=None):
        """forward(x, y) and the backward of its loss in one pass, each prior's backward issued
        on that prior's own stream right after its loss: the two priors are disjoint
        subgraphs of loss_l + loss_h (d/d loss_l = d/d loss_h = 1), so backpropagating each
        from its own root gives exactly the gradients of the sum -- and the LF prior's
        backward does not wait for the HF prior's forward (nor the HF backward for the LF
        forward) at a join before the loss.  `one`: a cached 0-dim ones tensor (the root
        gradient).  Returns a callable that builds (loss, (loss_l, loss_h)); call it after
        the streams are joined (the enclosing streams.concurrent() region's exit)."""
        loss_l, loss_h = self._priors(x, y, draws, one)

        def total():
            with torch.no_grad():
                return add_losses(loss_l.detach(), loss_h.detach()), (loss_l.detach(),
                                                                      loss_h.detach())
        return total

    def _priors(self, x, y, draws, one):
        """The body forward() and forward_backward() share (maskgit.py:155-192): encode with
        the frozen stage1, mask both token sequences, run the HF prior on a side stream
        concurrently with the LF prior, each to its masked cross-entropy.  `one` given: each
        prior's backward from its own loss right after it, and the side stream is left for
        the enclosing concurrent region to join; `one` None: forward only, joined here."""
        self.encoder_l.eval()
        self.vq_model_l.eval()
        self.encoder_h.eval()
        self.vq_model_h.eval()
        dr = draws or {}
        s_l, s_h = self.encode_tokens(x)
        s_l_M, keep_l = self._randomly_mask_tokens(s_l, self.mask_token_ids["lf"], x.device,
                                                   dr.get("ratio_l"), dr.get("rand_l"))
        s_h_M, keep_h = self._randomly_mask_tokens(s_h, self.mask_token_ids["hf"], x.device,
                                                   dr.get("ratio_h"), dr.get("rand_h"))
        self.transformer_l._class_rand = dr.get("cls_l")
        self.transformer_h._class_rand = dr.get("cls_h")
        try:
            with streams.branch(x.device) as br:  # HF transformer concurrently with LF
                br.inputs(y, s_l_M, s_h_M, s_h, keep_h, *(() if one is None else (one,)))
                with wgrad.tag("prior_h"):  # its weight gradients: one grouped launch
                    loss_h = self._prior_loss(self.transformer_h, y, (s_l_M, s_h_M), s_h, keep_h,
                                              one)
                    if one is not None:
                        torch.autograd.backward(loss_h, one)
                br.outputs(loss_h)
            with wgrad.tag("prior_l"):
                loss_l = self._prior_loss(self.transformer_l, y, (s_l_M,), s_l, keep_l, one)
                if one is not None:
                    torch.autograd.backward(loss_l, one)
            if one is None:
                br.join()
        finally:
            self.transformer_l._class_rand = self.transformer_h._class_rand = None
        return loss_l, loss_h

    def _prior_loss(self, tf, y, s_in, target, keep, one):
        """masked_cross_entropy(masked_prediction(tf, y, *s_in), target, keep) (maskgit.py:
        180-191).  With `one` (the root gradient of forward_backward) and no guidance mixing,
        the tied logits, the loss and its gradient down to the head output run as one fused
        pass (bidirectional_transformer.tied_logits_ce): the logits never reach memory."""
        if one is not None and bt.TIED_CE_FUSED and (y is None or self.cfg_scale == 1.0):
            h = tf._embed_hf(*s_in, y) if tf.kind == "hf" else tf._embed_lf(s_in[0], y)
            W = tf.tok_emb_h.weight if tf.kind == "hf" else tf.tok_emb_l.weight
            if bt.tied_ce_supported(h, W, tf.codebook_size):
                return bt.tied_logits_ce(h, W, tf.bias, tf.codebook_size, target, keep, one)
            logits = bt._TiedLogits.apply(h, W, tf.bias, tf.codebook_size)
            return masked_cross_entropy(logits, target, keep)
        return masked_cross_entropy(self.masked_prediction(tf, y, *s_in), target, keep)

    def _randomly_mask_tokens(self, s, mask_token_id, device, ratio=None, rand=None):
        """maskgit.py:194-216 on device; returns (s_M, mask) with mask=True for kept tokens.
        ratio (b,) / rand (b, n): injected draws (tests), else the device RNG."""
        site = self._site_mask_l if s.shape[1] == self.num_tokens_l else self._site_mask_h
        if ratio is not None:
            ratio = torch.as_tensor(ratio, dtype=torch.float64).to(device)
        if rand is not None:
            rand = torch.as_tensor(rand, dtype=torch.float32).to(device)
        return mask_tokens(s, mask_token_id, site, ratio=ratio, rand=rand)

    def gamma_func(self, mode="cosine"):
        """maskgit.py:218-228."""
        if mode == "linear":
            return lambda r: 1 - r
        if mode == "cosine":
            return lambda r: np.cos(r * np.pi / 2)
        if mode == "square":
            return lambda r: 1 - r ** 2
        if mode == "cubic":
            return lambda r: 1 - r ** 3
        raise NotImplementedError

    def create_input_tokens_normal(self, num, num_tokens, mask_token_ids, device):
        """maskgit.py:230-236."""
        return full_tokens((num, num_tokens), mask_token_ids, device)

    def mask_by_random_topk(self, mask_len, probs, temperature=1.0, device="cpu"):
        """maskgit.py:238-267: bool masking of exactly mask_len lowest-confidence tokens
        per row, confidence = log(probs + 1e-5) + temperature * Gumbel noise."""
        k = int(mask_len.unique().item()) if torch.is_tensor(mask_len) else int(mask_len)
        return maskgit_remask(probs.float(), k, temperature, site=self._site_sample,
                              want_masking=True)

    def sample_tokens(self, transformer, class_condition, mask_id, *s_in, gumbel=None,
                      want_logits=False, first=True):
        """The categorical draw of one decoding step (maskgit.py:302-326): masked_prediction's
        logits -> Categorical(logits).sample() -> (sampled with known tokens kept,
        p(sampled)).  Without guidance (cfg 1 or no class) the prior draws straight from its
        head (BidirectionalTransformer.sample); with guidance the two forwards' logits are
        mixed first."""
        if class_condition is None or self.cfg_scale == 1.0:
            return transformer.sample(*s_in, class_condition=class_condition, mask_id=mask_id,
                                      gumbel=gumbel, site=self._site_sample,
                                      want_logits=want_logits, first=first)
        logits = self.masked_prediction(transformer, class_condition, *s_in)
        out = maskgit_sample(logits, s_in[-1], mask_id, gumbel=gumbel, site=self._site_sample)
        return out + (logits,) if want_logits else out

    def _decode_pass(self, sample_call, s, mask_id, T, temperature, unknown0, gamma):
        """One of first_pass / second_pass: T steps of (draw -> re-mask)."""
        n0 = int(unknown0.max().item()) if torch.is_tensor(unknown0) else int(unknown0)
        for t in range(T):
            ratio = 1.0 * (t + 1) / T
            k = mask_len(n0, gamma(ratio))
            sampled, selp = sample_call(s, t == 0)  # later steps reuse the packed weights
            s = maskgit_remask(selp, k, temperature * (1.0 - ratio), sampled, mask_id,
                               site=self._site_sample)
        return s

    def first_pass(self, s_l: torch.Tensor, unknown_number_in_the_beginning_l,
                   class_condition: Union[torch.Tensor, None], gamma: Callable, device):
        """maskgit.py:294-355."""
        mask_id = self.mask_token_ids["lf"]
        return self._decode_pass(
            lambda s, first: self.sample_tokens(self.transformer_l, class_condition, mask_id, s,
                                                first=first), s_l,
            mask_id, self.T["lf"], self.choice_temperature_l,
            unknown_number_in_the_beginning_l, gamma)

    def second_pass(self, s_l: torch.Tensor, s_h: torch.Tensor, unknown_number_in_the_beginning_h,
                    class_condition: Union[torch.Tensor, None], gamma: Callable, device):
        """maskgit.py:357-411."""
        mask_id = self.mask_token_ids["hf"]
        return self._decode_pass(
            lambda s, first: self.sample_tokens(self.transformer_h, class_condition, mask_id, s_l,
                                                s, first=first),
            s_h, mask_id, self.T["hf"], self.choice_temperature_h,
            unknown_number_in_the_beginning_h, gamma)

    @torch.no_grad()
    def iterative_decoding(self, num=1, mode="cosine", class_index=None, device="cpu",
                           after_lf=None):
        """maskgit.py:413-446 -> (s_l (num, n), s_h (num, m)) int64, on `device`.  Every
        step stays on the device; the only host values are the per-step mask lengths,
        known in advance (all tokens start masked).  after_lf(s_l), if given, is called once
        the LF tokens are final, before the HF pass (GraphedSampler forks the LF decoder
        onto a side stream there); the HF pass only reads s_l."""
        s_l = self.create_input_tokens_normal(num, self.num_tokens_l, self.mask_token_ids["lf"],
                                              device)
        s_h = self.create_input_tokens_normal(num, self.num_tokens_h, self.mask_token_ids["hf"],
                                              device)
        gamma = self.gamma_func(mode)
        class_condition = (torch.full((num, 1), int(class_index), dtype=torch.int32, device=device)
                           if class_index is not None else None)
        s_l = self.first_pass(s_l, self.num_tokens_l, class_condition, gamma, device)
        if after_lf is not None:
            after_lf(s_l)
        s_h = self.second_pass(s_l, s_h, self.num_tokens_h, class_condition, gamma, device)
        return s_l, s_h

    def decode_token_ind_to_timeseries(self, s: torch.Tensor, frequency: str,
                                       return_representations: bool = False):
        """maskgit.py:448-477."""
        frequency = frequency.lower()
        assert frequency in ["lf", "hf"]
        vq_model = self.vq_model_l if frequency == "lf" else self.vq_model_h
        decoder = self.decoder_l if frequency == "lf" else self.decoder_h
        H_prime = self.H_prime_l if frequency == "lf" else self.H_prime_h
        W_prime = self.W_prime_l if frequency == "lf" else self.W_prime_h
        with torch.no_grad():
            # project_out is Identity (codebook_dim == dim), so the lookup goes straight
            # into the decoder's (b, c, h, w) layout
            zq = codebook_gather_nchw(s, vq_model._codebook.embed, H_prime, W_prime)
            xhat = decoder(zq)
        if return_representations:
            return xhat, zq
        return xhat
