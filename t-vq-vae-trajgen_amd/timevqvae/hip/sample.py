"""MaskGIT sampling ops on the HIP path (include/tvq.h §MaskGIT sampling).

maskgit_sample + maskgit_remask together are one step of first_pass / second_pass
(reference maskgit.py:294-411); codebook_gather_nchw is the codebook lookup of
decode_token_ind_to_timeseries (maskgit.py:461-469)."""
import numpy as np
import torch

from . import rng
from ._native import call, ptr, stream_ptr, value


def mask_len(unknown0: int, mask_ratio: float) -> int:
    """floor(unknown0 * mask_ratio) in float32, clipped at 0 (maskgit.py:328-333)."""
    return max(0, int(np.floor(np.float32(unknown0) * np.float32(mask_ratio))))


def full_tokens(shape, value, device):
    """torch.full(shape, value, int64) on the HIP path (tvq_fill_i64): the all-masked token
    rows of MaskGIT.create_input_tokens_normal (maskgit.py:230-236)."""
    t = torch.empty(shape, dtype=torch.int64, device=device)
    if t.is_cuda:
        call("tvq_fill_i64", ptr(t), t.numel(), int(value), stream_ptr())
    else:
        t.fill_(int(value))
    return t


def maskgit_sample(logits, s, mask_id, gumbel=None, site=0):
    """(sampled ids with known tokens kept, p(sampled) with +inf for known tokens).

    The draw is Categorical(logits).sample() as torch runs it -- torch.multinomial's
    n_sample = 1 exponential race, argmax_k l_k + Gumbel_k (maskgit.py:307-315) -- with the
    Gumbel noise from the device seed's counter hash, or `gumbel` (B, n, K) when given."""
    B, n, K = logits.shape
    sb, sn, sk = logits.stride()
    if sk != 1:
        raise ValueError("maskgit_sample: logits must be contiguous along the code axis")
    s = s.contiguous()
    sampled = torch.empty_like(s)
    selp = torch.empty((B, n), device=logits.device, dtype=torch.float32)
    seed = rng.seed_tensor(logits.device) if gumbel is None else None
    off = rng.call_offset(site) if gumbel is None else 0
    call("tvq_maskgit_sample", ptr(logits), sb, sn, B, n, K, ptr(s), int(mask_id),
         ptr(gumbel.contiguous() if gumbel is not None else None), ptr(seed), off, ptr(sampled),
         ptr(selp), stream_ptr())
    return sampled, selp


_tls_ws = {}


def tied_logits_sample(h, W, bias, K, s, mask_id, gumbel=None, site=0, want_logits=False):
    """maskgit_sample(h @ W[:K]^T + bias[:, :K], s, mask_id) in one pass: the tied logits of
    the prior's head (bidirectional_transformer.py:186-191) computed on MFMA and consumed by
    the race in registers, never written to memory (include/tvq.h tvq_tied_logits_sample).
    h (B, n, D) with D 64 or 128; bias (n, ldb >= K).  want_logits: also return the logits
    the draw used (tests)."""
    B, n, D = h.shape
    M = B * n
    h2 = h.reshape(M, D).contiguous()
    s = s.contiguous()
    dev = h.device
    nb = bias.shape[0]
    key = (dev, K, D, nb)
    ws = _tls_ws.get(key)
    if ws is None:
        nbytes = value("tvq_tied_logits_sample_workspace", K, D, nb)
        if nbytes < 0:
            raise ValueError("tied_logits_sample: unsupported shape")
        ws = torch.empty((nbytes + 15) // 16 * 4, device=dev, dtype=torch.float32)
        _tls_ws[key] = ws
    sampled = torch.empty_like(s)
    selp = torch.empty((B, n), device=dev, dtype=torch.float32)
    logits = torch.empty((B, n, K), device=dev, dtype=torch.float32) if want_logits else None
    seed = rng.seed_tensor(dev) if gumbel is None else None
    off = rng.call_offset(site) if gumbel is None else 0
    call("tvq_tied_logits_sample", ptr(h2), M, D, ptr(W.contiguous()), K, ptr(bias), nb,
         bias.stride(0), ptr(s), int(mask_id),
         ptr(gumbel.contiguous() if gumbel is not None else None), ptr(seed), off,
         ptr(sampled), ptr(selp), ptr(logits), ptr(ws), stream_ptr())
    return (sampled, selp, logits) if want_logits else (sampled, selp)


def maskgit_remask(selp, k, temperature, sampled=None, mask_id=0, u_gumbel=None, site=0,
                   want_masking=False):
    """Re-mask the k lowest-confidence tokens per row.  Returns s_out (if sampled given)
    and/or the bool masking (want_masking)."""
    B, n = selp.shape
    dev = selp.device
    s_out = torch.empty_like(sampled) if sampled is not None else None
    masking = torch.empty((B, n), device=dev, dtype=torch.uint8) if want_masking else None
    seed = rng.seed_tensor(dev) if u_gumbel is None else None
    off = rng.call_offset(site) if u_gumbel is None else 0
    call("tvq_maskgit_remask", ptr(selp.contiguous()), B, n, int(k), float(temperature),
         ptr(u_gumbel.contiguous() if u_gumbel is not None else None), ptr(seed), off,
         ptr(sampled), int(mask_id), ptr(s_out), ptr(masking), stream_ptr())
    if want_masking:
        return (s_out, masking.bool()) if s_out is not None else masking.bool()
    return s_out


def codebook_gather_nchw(s, E, H, W):
    """E[s] laid out (b, d, H, W) for the decoder (s: (b, H*W) int64, E: (K, d))."""
    B, P = s.shape
    K, D = E.shape
    if P != H * W:
        raise ValueError("codebook_gather_nchw: token count != H*W")
    out = torch.empty((B, D, H, W), device=E.device, dtype=torch.float32)
    call("tvq_codebook_gather_nchw", ptr(s.contiguous()), B, P, D, ptr(E.contiguous()), ptr(out),
         stream_ptr())
    return out
