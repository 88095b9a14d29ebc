"""Stage1 VQ-VAE trainer — the reference trainers/stage1.py contract without Lightning.

Same constructor (input_length, in_channels, config), module attributes
(encoder_l/h, vq_model_l/h, decoder_l/h; state_dict keys identical),
forward(batch, batch_idx, return_x_rec) and training_step(batch, batch_idx) ->
loss_hist with the reference's logged scalar names (stage1.py:183-196).
One fused STFT kernel produces both encoder inputs and both targets
(stage1.py:101-113 + vq_vae.py:179-180).
"""
import torch
import torch.nn as nn

from ..hip import streams, wgrad
from ..hip.conv import wgrad_deferred
from ..hip.loss import l1_loss, loss_sums, mse_loss
from ..hip.optim import FusedAdamW
from ..utils.checkpoint import adapt_state_dict, read_state_dict, save_checkpoint
from ..hip.signal import stft_encode
from ..models import VectorQuantize, VQVAEDecoder, VQVAEEncoder
from ..utils import (compute_downsample_rate, linear_warmup_cosine_annealingLR, quantize,
                     zero_pad_high_freq, zero_pad_low_freq)


class Stage1(nn.Module):
    def __init__(self, input_length: int, in_channels: int, config: dict, **kwargs):
        super().__init__()
        self.input_length = input_length
        self.config = config
        self.n_fft = config["VQ-VAE"]["n_fft"]
        init_dim = config["encoder"]["init_dim"]
        hid_dim = config["encoder"]["hid_dim"]
        dw_l = config["encoder"]["downsampled_width"]["lf"]
        dw_h = config["encoder"]["downsampled_width"]["hf"]
        rate_l = compute_downsample_rate(input_length, self.n_fft, dw_l)
        rate_h = compute_downsample_rate(input_length, self.n_fft, dw_h)
        n_res = config["encoder"]["n_resnet_blocks"]
        self.encoder_l = VQVAEEncoder(init_dim, hid_dim, 2 * in_channels, rate_l, n_res,
                                      zero_pad_high_freq, self.n_fft, frequency_indepence=False)
        self.encoder_h = VQVAEEncoder(init_dim, hid_dim, 2 * in_channels, rate_h, n_res,
                                      zero_pad_low_freq, self.n_fft, frequency_indepence=False)
        self.vq_model_l = VectorQuantize(hid_dim, config["VQ-VAE"]["codebook_sizes"]["lf"],
                                         **config["VQ-VAE"])
        self.vq_model_h = VectorQuantize(hid_dim, config["VQ-VAE"]["codebook_sizes"]["hf"],
                                         **config["VQ-VAE"])
        n_res_d = config["decoder"]["n_resnet_blocks"]
        self.decoder_l = VQVAEDecoder(init_dim, hid_dim, 2 * in_channels, rate_l, n_res_d,
                                      input_length, zero_pad_high_freq, self.n_fft, in_channels,
                                      frequency_indepence=False)
        self.decoder_h = VQVAEDecoder(init_dim, hid_dim, 2 * in_channels, rate_h, n_res_d,
                                      input_length, zero_pad_low_freq, self.n_fft, in_channels,
                                      frequency_indepence=False)
        self._sched = None
        self._opt = None

    def forward(self, batch, batch_idx, return_x_rec: bool = False):
        """stage1.py:89-168 (the validation-time plot is not reproduced)."""
        x, y = batch
        need_tgt = not return_x_rec
        s = stft_encode(x, enc_l=True, enc_h=True, tgt_l=need_tgt, tgt_h=need_tgt)
        # the HF branch runs on a side stream, concurrently with the LF branch
        with streams.branch(x.device, "s1hf") as br:
            br.inputs(s)
            hf = self._band("HF", s, return_x_rec)
            br.outputs(hf)
        lf = self._band("LF", s, return_x_rec)
        br.join()
        if return_x_rec:
            return lf[0] + hf[0]
        return self._assemble({"LF": lf, "HF": hf})

    def _band(self, band, s, return_x_rec=False):
        """One frequency band (stage1.py:115-166): encoder -> VQ -> decoder (-> loss).
        Returns (xhat, recons_loss, vq_loss, perplexity)."""
        if band == "LF":
            enc, vq, dec, tgt, loss_fn = self.encoder_l, self.vq_model_l, self.decoder_l, "tgt_l", mse_loss
            z = enc.encode_timefreq(s["enc_l"])
        else:
            enc, vq, dec, tgt, loss_fn = self.encoder_h, self.vq_model_h, self.decoder_h, "tgt_h", l1_loss
            z = enc.encode_timefreq(s["enc_h"])
        z_q, _, vq_loss, perplexity = quantize(z, vq)
        xhat = dec(z_q)
        rec = None if return_x_rec else loss_fn(s[tgt], xhat)
        return xhat, rec, vq_loss, perplexity

    def _ones(self, t):
        """A cached ones tensor of t's shape (made outside graph capture, reused)."""
        cache = self.__dict__.setdefault("_ones_cache", {})
        key = (tuple(t.shape), t.device)
        if key not in cache:
            cache[key] = torch.ones(t.shape, device=t.device, dtype=t.dtype)
        return cache[key]

    @staticmethod
    def _assemble(parts):
        recons_loss = {"LF.time": parts["LF"][1], "HF.time": parts["HF"][1]}
        vq_losses = {"LF": parts["LF"][2], "HF": parts["HF"][2]}
        perplexities = {"LF": parts["LF"][3], "HF": parts["HF"][3]}
        return recons_loss, vq_losses, perplexities

    def forward_backward(self, batch, batch_idx=0, bands=("HF", "LF")):
        """training_step + backward of its loss, with each band's forward AND backward on
        its own stream inside streams.concurrent() (both fork off the current stream).
        The two bands are disjoint subgraphs of the loss sum, so backpropagating
        (recons + vq loss) per band gives exactly the gradients of loss.sum().  Returns a
        callable that builds training_step's dict; call it after the region's join.
        `bands` (diagnosis: bench.py's TVQ_BENCH_BANDS times one band alone) must name both
        bands for a training step; a single band returns a zero loss."""
        x, y = batch
        s = stft_encode(x, enc_l=True, enc_h=True, tgt_l=True, tgt_h=True)
        parts = {}
        for band in ("HF", "LF"):
            if band not in bands:
                continue
            with streams.branch(x.device, "s1" + band.lower()) as br:
                br.inputs(s)
                part = self._band(band, s)
                # conv weight-gradient split sums and Linear weight gradients batched at
                # the band's end
                with wgrad_deferred(), wgrad.grouped():
                    # d(recons + vq_loss).sum() = 1 for both roots: backward from the two
                    # roots with cached ones (no add / sum / ones_like launches)
                    torch.autograd.backward((part[1], part[2]["loss"]),
                                            (self._ones(part[1]), self._ones(part[2]["loss"])))
                parts[band] = part
                br.outputs(part)
        if self._sched is not None:
            self._sched.step()
        if len(parts) < 2:
            return lambda: {"loss": torch.zeros((), device=x.device)}
        return lambda: self._loss_hist(*self._assemble(parts), fused=True)

    def training_step(self, batch, batch_idx):
        """stage1.py:170-198: loss and the logged scalars; steps the LR scheduler."""
        recons_loss, vq_losses, perplexities = self.forward(batch, batch_idx)
        if self._sched is not None:
            self._sched.step()
        return self._loss_hist(recons_loss, vq_losses, perplexities)

    @staticmethod
    def _loss_hist(recons_loss, vq_losses, perplexities, fused=False):
        """fused: the sums for logging only (after forward_backward), one launch"""
        rl, rh = recons_loss["LF.time"], recons_loss["HF.time"]
        if fused:
            loss, rsum = loss_sums(rl, rh, vq_losses["LF"]["loss"], vq_losses["HF"]["loss"])
        else:
            loss = (rl + rh) + vq_losses["LF"]["loss"] + vq_losses["HF"]["loss"]
            rsum = rl + rh
        return {
            "loss": loss,
            "recons_loss.time": rsum,
            "recons_loss.LF.time": recons_loss["LF.time"],
            "recons_loss.HF.time": recons_loss["HF.time"],
            "commit_loss.LF": vq_losses["LF"]["commit_loss"],
            "commit_loss.HF": vq_losses["HF"]["commit_loss"],
            "perplexity.LF": perplexities["LF"],
            "perplexity.HF": perplexities["HF"],
        }

    @torch.no_grad()
    def validation_step(self, batch, batch_idx):
        self.eval()
        recons_loss, vq_losses, perplexities = self.forward(batch, batch_idx)
        return {"loss": (recons_loss["LF.time"] + recons_loss["HF.time"]),
                "recons_loss.LF.time": recons_loss["LF.time"],
                "recons_loss.HF.time": recons_loss["HF.time"],
                "perplexity.LF": perplexities["LF"], "perplexity.HF": perplexities["HF"]}

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location="cpu", input_length=None,
                             in_channels=None, config=None, strict=True, weights_only=True,
                             **kwargs):
        """Lightning-style loader (maskgit.py:52-59): a reference `stage1.ckpt`
        ({'state_dict': ...}) or a bare state_dict; tensors only (utils/checkpoint.py)."""
        sd = read_state_dict(checkpoint_path, map_location, weights_only)
        model = cls(input_length, in_channels, config, **kwargs)
        model.load_state_dict(adapt_state_dict(sd, model), strict=strict)
        return model

    def save_checkpoint(self, path, **extra):
        save_checkpoint(self, path, **extra)

    def configure_optimizers(self):
        """stage1.py:229-236: AdamW(lr) + linear warmup / cosine annealing."""
        opt = FusedAdamW(self.parameters(), lr=self.config["exp_params"]["lr"])
        sch = linear_warmup_cosine_annealingLR(opt, self.config["trainer_params"]["max_steps"]["stage1"],
                                               self.config["exp_params"]["linear_warmup_rate"])
        self._opt, self._sched = opt, sch
        return {"optimizer": opt, "lr_scheduler": sch}
