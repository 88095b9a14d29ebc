"""n_fft=4 STFT front end and decoder iSTFT tail on the HIP path."""
import torch

from ._native import call, ptr, stream_ptr

BAND = {"lf": 0, "hf": 1, "all": 2}


def stft_encode(x, raw=False, enc_l=False, enc_h=False, tgt_l=False, tgt_h=False):
    """One pass over x (B,C,T): returns dict of the requested outputs (no grad: data path).

    raw   time_to_timefreq(x)                              (B,2C,3,T+1)
    enc_l zero_pad_high_freq(raw, copy=True)               (B,2C,3,T+1)
    enc_h zero_pad_low_freq(raw, copy=True)                (B,2C,3,T+1)
    tgt_l interp(istft(zero_pad_high_freq(raw)), T)        (B,C,T)
    tgt_h interp(istft(zero_pad_low_freq(raw)), T)         (B,C,T)
    """
    x = x.detach().contiguous()
    B, C, T = x.shape
    img = lambda: torch.empty((B, 2 * C, 3, T + 1), device=x.device, dtype=torch.float32)
    ser = lambda: torch.empty((B, C, T), device=x.device, dtype=torch.float32)
    out = {}
    if raw: out["raw"] = img()
    if enc_l: out["enc_l"] = img()
    if enc_h: out["enc_h"] = img()
    if tgt_l: out["tgt_l"] = ser()
    if tgt_h: out["tgt_h"] = ser()
    call("tvq_stft_encode", ptr(x), B, C, T, ptr(out.get("raw")), ptr(out.get("enc_l")),
         ptr(out.get("enc_h")), ptr(out.get("tgt_l")), ptr(out.get("tgt_h")), stream_ptr())
    return out


class _ISTFTDecode(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, C, band, Tout):
        h = h.contiguous()
        B, _, _, W = h.shape
        y = torch.empty((B, C, Tout), device=h.device, dtype=torch.float32)
        call("tvq_istft_decode", ptr(h), B, C, W, band, Tout, ptr(y), stream_ptr())
        ctx.cfg = (B, C, W, band, Tout)
        return y

    @staticmethod
    def backward(ctx, gy):
        B, C, W, band, Tout = ctx.cfg
        g = gy.contiguous()
        dh = torch.empty((B, 2 * C, 3, W), device=g.device, dtype=torch.float32)
        call("tvq_istft_decode_bwd", ptr(g), B, C, W, band, Tout, ptr(dh), stream_ptr())
        return dh, None, None, None


def istft_decode(h, C, band, Tout):
    """interp(istft(band_mask(h)), Tout): h (B,2C,3,W) -> (B,C,Tout); band 'lf'|'hf'|'all'."""
    return _ISTFTDecode.apply(h, int(C), BAND[band] if isinstance(band, str) else int(band),
                              int(Tout))
