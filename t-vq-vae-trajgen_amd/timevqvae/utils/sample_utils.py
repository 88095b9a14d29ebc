"""Batched sampling helpers -- same API as the reference timevqvae/utils/sample_utils.py
(unconditional_sample / conditional_sample, sample_utils.py:5-88; the plotting helper is
not on the path).  MaskGIT.iterative_decoding and decode_token_ind_to_timeseries run on
the HIP path; each batch reaches the host by an asynchronous copy into pinned memory."""
import os

import torch

from ..hip.loss import add_losses


def _batch_sizes(n_samples: int, batch_size: int):
    """Sizes of the sampling batches: full batches, then the remainder (if any)."""
    full, rest = divmod(int(n_samples), int(batch_size))
    return [int(batch_size)] * full + ([rest] if rest else [])


@torch.no_grad()
def unconditional_sample(maskgit, n_samples: int, device, class_index=None, batch_size=32,
                         return_representations=False):
    """Same contract as the reference (sample_utils.py:5-64): (x_l, x_h, x) on the host,
    and with return_representations also the decoder inputs (quantize_l, quantize_h).

    Each batch's decoded LF / HF series (and latents) are copied asynchronously into
    preallocated pinned host buffers (non_blocking device->host copies on the stream; one
    synchronisation at the end), so device memory stays bounded by one batch, as the
    reference's per-batch `.cpu()` keeps it, without a host round trip per batch."""
    device = torch.device(device)
    sizes = _batch_sizes(n_samples, batch_size)
    if not sizes:
        raise ValueError("unconditional_sample: n_samples must be positive")
    host = None
    row = 0
    pin = device.type == "cuda"
    for b in sizes:
        s_l, s_h = maskgit.iterative_decoding(num=b, device=device, class_index=class_index)
        parts = []
        for s, band in ((s_l, "lf"), (s_h, "hf")):
            out = maskgit.decode_token_ind_to_timeseries(s, band, return_representations)
            parts.append(out if return_representations else (out, None))
        (x_l, q_l), (x_h, q_h) = parts
        outs = [x_l, x_h] + ([q_l, q_h] if return_representations else [])
        if host is None:  # shapes are known after the first batch
            host = [torch.empty((n_samples,) + tuple(t.shape[1:]), dtype=t.dtype, pin_memory=pin)
                    for t in outs]
        for h, t in zip(host, outs):
            h[row:row + b].copy_(t, non_blocking=pin)
        row += b
    if pin:
        torch.cuda.current_stream(device).synchronize()
    x_l, x_h = host[0], host[1]
    series = (x_l, x_h, x_l + x_h)  # summed on the host, as the reference does
    if return_representations:
        return series, (host[2], host[3])
    return series


@torch.no_grad()
def conditional_sample(maskgit, n_samples: int, device, class_index: int, batch_size=32,
                       return_representations=False):
    """class_index: starting from 0 (sample_utils.py:70-88)."""
    return unconditional_sample(maskgit, n_samples, device, class_index, batch_size,
                                return_representations)


class GraphedSampler:
    """One sampling batch -- MaskGIT iterative decoding (maskgit.py:413-446), LF/HF decoding
    (maskgit.py:448-477) and optionally the FidelityEnhancer (sampler.py:156-169) --
    captured once as a hipGraph and replayed per batch.

    Every step of the batch already runs on the device with fixed shapes (the mask
    lengths are host constants, sampling noise is the counter hash of the device seed), so
    the graph holds the whole batch; the device seed advances inside it, so each replay
    draws a fresh batch, equal to the eager `rng.advance(); iterative_decoding(...)` from
    the same seed.  `sample()` returns (x_l, x_h, x[, x_R]) device tensors that the next
    replay overwrites (clone them to keep)."""

    def __init__(self, maskgit, num: int, device, class_index=None, fidelity_enhancer=None,
                 warmup: int = 2):
        from ..hip import rng
        from ..hip.graph import StepGraph
        self.maskgit, self.num, self.device = maskgit, num, torch.device(device)
        self.class_index, self.fe = class_index, fidelity_enhancer
        maskgit.eval()
        if fidelity_enhancer is not None:
            fidelity_enhancer.eval()

        from ..hip.conv import PackCache
        # the convs' packed weights: repacked by a few batched launches at the start of each
        # replay instead of one pack launch per conv (the weights are fixed within a batch)
        self.packs = PackCache(self.device)
        # the LF decoder needs only the final LF tokens: it runs on a side stream while the
        # HF prior's pass and the HF decoder run (TVQ_SAMPLER_OVERLAP=0: one stream)
        overlap = self.device.type == "cuda"
        self._side = torch.cuda.Stream(self.device) if overlap else None

        def batch():
            with torch.no_grad(), self.packs.scope():
                rng.advance(self.device)
                held = {}

                def after_lf(s_l):
                    if self._side is None:
                        return
                    self._side.wait_stream(torch.cuda.current_stream(self.device))
                    with torch.cuda.stream(self._side):
                        held["x_l"] = maskgit.decode_token_ind_to_timeseries(s_l, "lf")

                s_l, s_h = maskgit.iterative_decoding(num=num, device=self.device,
                                                      class_index=class_index,
                                                      after_lf=after_lf)
                x_h = maskgit.decode_token_ind_to_timeseries(s_h, "hf")
                if self._side is not None:
                    torch.cuda.current_stream(self.device).wait_stream(self._side)
                    x_l = held["x_l"]
                else:
                    x_l = maskgit.decode_token_ind_to_timeseries(s_l, "lf")
                out = (x_l, x_h, add_losses(x_l, x_h))  # one HIP add (tvq_sum4)
                if fidelity_enhancer is not None:
                    out = out + (fidelity_enhancer(out[2]),)
                return out

        self.graph = StepGraph([batch], warmup=warmup).capture()

    def sample(self):
        return self.graph.replay()[0]
