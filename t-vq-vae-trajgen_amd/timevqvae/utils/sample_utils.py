"""Batched sampling helpers -- same API as the reference timevqvae/utils/sample_utils.py
(unconditional_sample / conditional_sample, sample_utils.py:5-88; the plotting helper is
not on the path).  MaskGIT.iterative_decoding and decode_token_ind_to_timeseries run on
the HIP path; results are moved to the host per batch, as in the reference."""
import torch


@torch.no_grad()
def unconditional_sample(maskgit, n_samples: int, device, class_index=None, batch_size=32,
                         return_representations=False):
    n_iters = n_samples // batch_size
    is_residual_batch = False
    if n_samples % batch_size > 0:
        n_iters += 1
        is_residual_batch = True
    x_new_l, x_new_h, x_new = [], [], []
    quantize_new_l, quantize_new_h = [], []
    for i in range(n_iters):
        b = batch_size
        if (i + 1 == n_iters) and is_residual_batch:
            b = n_samples - ((n_iters - 1) * batch_size)
        embed_ind_l, embed_ind_h = maskgit.iterative_decoding(num=b, device=device,
                                                              class_index=class_index)
        if return_representations:
            x_l, quantize_l = maskgit.decode_token_ind_to_timeseries(embed_ind_l, "lf", True)
            x_h, quantize_h = maskgit.decode_token_ind_to_timeseries(embed_ind_h, "hf", True)
            x_l, quantize_l, x_h, quantize_h = x_l.cpu(), quantize_l.cpu(), x_h.cpu(), quantize_h.cpu()
            quantize_new_l.append(quantize_l)
            quantize_new_h.append(quantize_h)
        else:
            x_l = maskgit.decode_token_ind_to_timeseries(embed_ind_l, "lf").cpu()
            x_h = maskgit.decode_token_ind_to_timeseries(embed_ind_h, "hf").cpu()
        x_new_l.append(x_l)
        x_new_h.append(x_h)
        x_new.append(x_l + x_h)
    x_new_l = torch.cat(x_new_l)
    x_new_h = torch.cat(x_new_h)
    x_new = torch.cat(x_new)
    if return_representations:
        return (x_new_l, x_new_h, x_new), (torch.cat(quantize_new_l), torch.cat(quantize_new_h))
    return x_new_l, x_new_h, x_new


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

        def batch():
            with torch.no_grad():
                rng.advance(self.device)
                s_l, s_h = maskgit.iterative_decoding(num=num, device=self.device,
                                                      class_index=class_index)
                x_l = maskgit.decode_token_ind_to_timeseries(s_l, "lf")
                x_h = maskgit.decode_token_ind_to_timeseries(s_h, "hf")
                out = (x_l, x_h, x_l + x_h)
                if fidelity_enhancer is not None:
                    out = out + (fidelity_enhancer(out[2]),)
                return out

        self.graph = StepGraph([batch], warmup=warmup).capture()

    def sample(self):
        return self.graph.replay()[0]
