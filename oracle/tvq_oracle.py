"""TEST INFRASTRUCTURE ONLY — functional fp32 CPU restatement of the reference hot path.

Every function names the reference file:line it restates (paths relative to the
reference repo root, `timevqvae/...`).  The restatement is functional: it takes a
state_dict-shaped mapping of tensors (same keys as the reference module tree) and
returns outputs, so the same weights can be pushed through the product's HIP path
and through this oracle.  Pinned against tests/golden/*.npz, which were produced
by running the reference itself (tests/golden/make_golden.py).

Float work uses torch CPU fp32 (the reference's own arithmetic); the STFT/iSTFT
are written out as the explicit n_fft=4 DFT so the formula the HIP kernels follow
is visible here.  The transformer (x-transformers, absent from the image) is a
restatement from its published 1.3x behaviour: PARITY UNPINNED for T1 (see
DESIGN.md §Oracle).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------
# STFT / iSTFT, n_fft = 4, hop 1, periodic Hann, center+reflect, normalized
# ----------------------------------------------------------------------------
HANN4 = (0.0, 0.5, 1.0, 0.5)


def stft4(x: torch.Tensor) -> torch.Tensor:
    """time_to_timefreq (utils/train_utils.py:293-307): (B,C,T) -> (B,2C,3,T+1).

    Channel 2c+0 is the real part, 2c+1 the imaginary part of bin f (H axis).
    X[f,t] = 0.5 * sum_n w[n] xp[t+n] exp(-2*pi*i*f*n/4), xp = reflect-pad(x, 2).
    """
    B, C, T = x.shape
    xp = F.pad(x.reshape(B * C, 1, T), (2, 2), mode="reflect").reshape(B, C, T + 4)
    x1, x2, x3 = xp[..., 1:T + 2], xp[..., 2:T + 3], xp[..., 3:T + 4]
    re0 = 0.5 * (0.5 * x1 + x2 + 0.5 * x3)
    re1 = 0.5 * (-x2)
    im1 = 0.5 * (-0.5 * x1 + 0.5 * x3)
    re2 = 0.5 * (-0.5 * x1 + x2 - 0.5 * x3)
    zero = torch.zeros_like(re0)
    real = torch.stack([re0, re1, re2], dim=2)  # (B,C,3,T+1)
    imag = torch.stack([zero, im1, zero], dim=2)
    return torch.stack([real, imag], dim=2).reshape(B, 2 * C, 3, T + 1)


def istft4(xf: torch.Tensor, C: int) -> torch.Tensor:
    """timefreq_to_time (utils/train_utils.py:310-321): (B,2C,3,W) -> (B,C,W-1).

    irfft of each frame (imag of DC/Nyquist ignored), Hann synthesis window,
    overlap-add, division by the window envelope (1.25 at sample 0, else 1.5),
    center trim of 2 samples.
    """
    B, C2, H, W = xf.shape
    z = xf.reshape(B, C, 2, 3, W) * 2.0  # undo normalized=True
    X0r, X1r, X1i, X2r = z[:, :, 0, 0], z[:, :, 0, 1], z[:, :, 1, 1], z[:, :, 0, 2]
    y1 = (X0r - X2r - 2 * X1i) / 4  # frame sample n=1
    y2 = (X0r + X2r - 2 * X1r) / 4  # n=2
    y3 = (X0r - X2r + 2 * X1i) / 4  # n=3
    L = W - 1
    out = torch.zeros(B, C, L, dtype=xf.dtype)
    # sample i <- frames i+1 (n=1), i (n=2), i-1 (n=3)
    out += 0.5 * y1[..., 1:W]
    out += 1.0 * y2[..., 0:L]
    out[..., 1:] += 0.5 * y3[..., 0:L - 1]
    env = torch.full((L,), 1.5, dtype=xf.dtype)
    env[0] = 1.25
    return out / env


def band_lf(xf, copy=False):
    """zero_pad_high_freq (utils/train_utils.py:361-372)."""
    if copy:
        return xf[:, :, :1, :].expand(-1, -1, xf.shape[2], -1).contiguous()
    out = torch.zeros_like(xf)
    out[:, :, 0] = xf[:, :, 0]
    return out


def band_hf(xf, copy=False):
    """zero_pad_low_freq (utils/train_utils.py:375-386)."""
    if copy:
        return torch.cat([xf[:, :, 1:2], xf[:, :, 1:]], dim=2).contiguous()
    out = torch.zeros_like(xf)
    out[:, :, 1:] = xf[:, :, 1:]
    return out


def linear_interp(x, size):
    """F.interpolate(mode='linear', align_corners=False) (stage1.py:103-113, vq_vae.py:254)."""
    return F.interpolate(x, size, mode="linear")


def compute_downsample_rate(input_length, n_fft, downsampled_width):
    """utils/train_utils.py:413-418."""
    if input_length >= downsampled_width:
        return round(input_length / (np.log2(n_fft) - 1) / downsampled_width)
    return 1


# ----------------------------------------------------------------------------
# Encoder / decoder (models/vq_vae.py)
# ----------------------------------------------------------------------------
def snake(x, a):
    """SnakeActivation.forward (utils/train_utils.py:446-448): x + (1/a) sin(a x)^2."""
    return x + (1 / a) * torch.sin(a * x) ** 2


def encoder_plan(init_dim, hid_dim, num_channels, downsample_rate, n_res):
    """Layer list of VQVAEEncoder (vq_vae.py:154-167): ('enc'|'res', cin, cout)."""
    d = init_dim
    plan = [("enc", num_channels, d)]
    d *= 2
    for _ in range(int(round(np.log2(downsample_rate))) - 1):
        plan.append(("enc", d // 2, d))
        for _ in range(n_res):
            plan.append(("res", d, d))
        d *= 2
    plan.append(("res", d // 2, hid_dim))
    return plan


def decoder_plan(init_dim, hid_dim, num_channels, downsample_rate, n_res):
    """Layer list of VQVAEDecoder (vq_vae.py:226-252): ('res'|'dec'|'convt', cin, cout)."""
    L = int(round(np.log2(downsample_rate)))
    d = int(init_dim * 2 ** (L - 1)) if L != 0 else int(init_dim)
    plan = [("res", hid_dim, d)]
    for _ in range(L - 1):
        for _ in range(n_res):
            plan.append(("res", d, d))
        d //= 2
        plan.append(("dec", 2 * d, d))
    plan.append(("convt", d, num_channels))
    plan.append(("convt", num_channels, num_channels))
    return plan


class Ctx:
    """Carries training flag, dropout prob and the buffer updates of one pass."""

    def __init__(self, training, dropout_p=0.0, dropout_gen=None):
        self.training = training
        self.dropout_p = dropout_p
        self.gen = dropout_gen
        self.updates = {}
        # tests: code indices to use instead of the argmax (prefix -> (rows,) int64), e.g.
        # the HIP path's, so an fp32 near-tie that resolved the other way (z differs from
        # this restatement's by reassociation) does not decouple everything downstream;
        # vq_forward records each forced row's argmax and fp64 top-2 gap in `ind_check`
        self.forced_ind = {}
        self.ind_check = {}


def _bn(ctx, sd, p, x):
    """nn.BatchNorm2d/1d (momentum 0.1, eps 1e-5); running stats updated when training."""
    rm = sd[p + "running_mean"].clone()
    rv = sd[p + "running_var"].clone()
    y = F.batch_norm(x, rm, rv, sd[p + "weight"], sd[p + "bias"], ctx.training, 0.1, 1e-5)
    if ctx.training:
        ctx.updates[p + "running_mean"] = rm
        ctx.updates[p + "running_var"] = rv
        ctx.updates[p + "num_batches_tracked"] = sd[p + "num_batches_tracked"] + 1
    return y


def _dropout(ctx, x, p):
    """nn.Dropout (vq_vae.py:52): F.dropout (torch's bernoulli_ draw, the reference's own
    CPU cost); with an explicit generator, the same mask law drawn from it."""
    if not ctx.training or p == 0.0:
        return x
    if ctx.gen is None:
        return F.dropout(x, p, training=True)
    keep = (torch.rand(x.shape, generator=ctx.gen) >= p).to(x.dtype)
    return x * keep / (1 - p)


def enc_block(ctx, sd, p, x):
    """VQVAEEncBlock (vq_vae.py:65-92): replicate-pad Conv2d(3x4, s(1,2)) -> BN -> Snake."""
    x = F.pad(x, (1, 1, 1, 1), mode="replicate")
    x = F.conv2d(x, sd[p + "block.0.weight"], sd[p + "block.0.bias"], stride=(1, 2))
    x = _bn(ctx, sd, p + "block.1.", x)
    return snake(x, sd[p + "block.2.a"])


def res_block(ctx, sd, p, x):
    """ResBlock (vq_vae.py:13-62): proj(x) + Drop(Conv(Snake(BN(Conv(Snake(x))))))."""
    h = snake(x, sd[p + "convs.0.a"])
    h = F.conv2d(h, sd[p + "convs.1.weight"], sd[p + "convs.1.bias"], padding=(1, 1))
    h = _bn(ctx, sd, p + "convs.2.", h)
    h = snake(h, sd[p + "convs.3.a"])
    h = F.conv2d(h, sd[p + "convs.4.weight"], sd[p + "convs.4.bias"], padding=(1, 1))
    h = _dropout(ctx, h, ctx.dropout_p)
    if p + "proj.weight" in sd:
        x = F.conv2d(x, sd[p + "proj.weight"], sd[p + "proj.bias"])
    return x + h


def dec_block(ctx, sd, p, x):
    """VQVAEDecBlock (vq_vae.py:95-121): ConvTranspose2d(3x4, s(1,2), p(1,1)) -> BN -> Snake."""
    x = F.conv_transpose2d(x, sd[p + "block.0.weight"], sd[p + "block.0.bias"],
                           stride=(1, 2), padding=(1, 1))
    x = _bn(ctx, sd, p + "block.1.", x)
    return snake(x, sd[p + "block.2.a"])


def encoder_forward(ctx, sd, prefix, x, plan, band):
    """VQVAEEncoder.forward (vq_vae.py:174-188)."""
    C = x.shape[1]
    h = stft4(x)
    h = band(h, copy=True)
    for i, (kind, _, _) in enumerate(plan):
        p = f"{prefix}encoder.{i}."
        h = enc_block(ctx, sd, p, h) if kind == "enc" else res_block(ctx, sd, p, h)
    return h


def decoder_forward(ctx, sd, prefix, z, plan, band, x_channels, input_length):
    """VQVAEDecoder.forward (vq_vae.py:257-264)."""
    h = z
    for i, (kind, _, _) in enumerate(plan):
        p = f"{prefix}decoder.{i}."
        if kind == "res":
            h = res_block(ctx, sd, p, h)
        elif kind == "dec":
            h = dec_block(ctx, sd, p, h)
        else:
            h = F.conv_transpose2d(h, sd[p + "weight"], sd[p + "bias"], stride=(1, 2), padding=(1, 1))
    h = band(h)
    h = istft4(h, x_channels)
    h = linear_interp(h, input_length)
    return h + F.linear(h, sd[prefix + "linear.weight"], sd[prefix + "linear.bias"])


# ----------------------------------------------------------------------------
# Vector quantiser (models/vq.py)
# ----------------------------------------------------------------------------
def vq_dist(flat, embed):
    """dist = -(|x|^2 - 2 x.E^T + |E|^2), the reference's evaluation order (vq.py:210-214)."""
    et = embed.t()
    return -(flat.pow(2).sum(1, keepdim=True) - 2 * flat @ et + et.pow(2).sum(0, keepdim=True))


def vq_sample(dist, temp):
    """softmax_sample (vq.py:51-56): argmax at temp 0, else Categorical(logits=dist/temp)
    drawn from torch's CPU RNG (same draws as the reference under the same seed)."""
    if not temp:
        return dist.argmax(dim=-1)
    return torch.distributions.Categorical(logits=dist / temp).sample()


def vq_sample_gumbel(dist, temp, gumbel):
    """The HIP path's Gumbel-max form of the same distribution: argmax(dist/temp + g),
    g = -log(-log u) (vq.py:39-48 gumbel_sample); first index on ties.  Returns (idx,
    fp64 top-2 gap of the perturbed logits)."""
    z = dist / temp + gumbel
    z64 = dist.double() / temp + gumbel.double()
    top2 = torch.topk(z64, 2, dim=-1).values
    return z.argmax(dim=-1), (top2[:, 0] - top2[:, 1])


def vq_forward(ctx, sd, prefix, x, decay=0.8, eps=1e-5, svq_temp=None):
    """VectorQuantize.forward + EuclideanCodebook.forward (vq.py:197-251, 325-407).

    x: (B,N,D).  Returns (quantize, embed_ind, commit_loss, perplexity).
    Buffer updates (EMA, training only) go to ctx.updates.  svq_temp > 0 samples the
    indices (vq.py:216-222) from torch's RNG.
    """
    cb = prefix + "_codebook."
    embed = sd[cb + "embed"]
    K = embed.shape[0]
    flat = x.reshape(-1, x.shape[-1])
    dist = vq_dist(flat, embed)
    ind = vq_sample(dist, svq_temp)
    forced = ctx.forced_ind.get(prefix)
    if forced is not None:
        forced = forced.reshape(-1).to(ind.dtype)
        with torch.no_grad():
            d64 = vq_dist(flat.detach().double(), embed.detach().double())
            top2 = torch.topk(d64, 2, dim=-1).values
        ctx.ind_check[prefix] = (ind.clone(), forced, (top2[:, 0] - top2[:, 1]),
                                 flat.detach().double().pow(2).sum(1) +
                                 embed.detach().double().pow(2).sum(1).max())
        ind = forced
    onehot = F.one_hot(ind, K).to(x.dtype)
    q = F.embedding(ind, embed).reshape(x.shape)
    ind = ind.reshape(x.shape[:-1])
    commit = torch.zeros(())
    if ctx.training:
        n = onehot.sum(0)
        cs = sd[cb + "cluster_size"].detach().clone().mul_(decay).add_(n, alpha=1 - decay)
        esum = flat.detach().t() @ onehot
        ea = sd[cb + "embed_avg"].detach().clone().mul_(decay).add_(esum.t(), alpha=1 - decay)
        tot = cs.sum()
        cs_s = (cs + eps) / (tot + K * eps) * tot
        ctx.updates[cb + "cluster_size"] = cs
        ctx.updates[cb + "embed_avg"] = ea
        ctx.updates[cb + "embed"] = ea / cs_s.unsqueeze(1)
        q = x + (q - x).detach()
        commit = F.mse_loss(q.detach(), x)
    avg = onehot.mean(0)
    perp = torch.exp(-torch.sum(avg * torch.log(avg + 1e-10)))
    return q, ind, commit, perp


def quantize(ctx, sd, prefix, z):
    """utils/train_utils.py:338-358 (2-D latent): 'b c h w -> b (h w) c' and back."""
    B, C, H, W = z.shape
    zt = z.permute(0, 2, 3, 1).reshape(B, H * W, C)
    q, ind, commit, perp = vq_forward(ctx, sd, prefix, zt)
    return q.reshape(B, H, W, C).permute(0, 3, 1, 2), ind, commit, perp


# ----------------------------------------------------------------------------
# Stage1 (trainers/stage1.py)
# ----------------------------------------------------------------------------
class Stage1Spec:
    """Architecture of trainers/stage1.py:16-87 for a given config."""

    def __init__(self, input_length, in_channels, init_dim=4, hid_dim=128, n_res=2,
                 width_lf=8, width_hf=32, n_fft=4):
        self.T, self.C = input_length, in_channels
        self.rate_l = compute_downsample_rate(input_length, n_fft, width_lf)
        self.rate_h = compute_downsample_rate(input_length, n_fft, width_hf)
        nc = 2 * in_channels
        self.enc_l = encoder_plan(init_dim, hid_dim, nc, self.rate_l, n_res)
        self.enc_h = encoder_plan(init_dim, hid_dim, nc, self.rate_h, n_res)
        self.dec_l = decoder_plan(init_dim, hid_dim, nc, self.rate_l, n_res)
        self.dec_h = decoder_plan(init_dim, hid_dim, nc, self.rate_h, n_res)


def stage1_targets(x):
    """stage1.py:101-113: LF/HF targets via STFT band split and iSTFT."""
    B, C, T = x.shape
    xf = stft4(x)
    x_l = linear_interp(istft4(band_lf(xf), C), T)
    x_h = linear_interp(istft4(band_hf(xf), C), T)
    return x_l, x_h


def stage1_forward(ctx, sd, spec, x, return_x_rec=False):
    """Stage1.forward (stage1.py:89-168) + the loss of training_step (stage1.py:170-176)."""
    x_l, x_h = stage1_targets(x)
    z_l = encoder_forward(ctx, sd, "encoder_l.", x, spec.enc_l, band_lf)
    zq_l, s_l, commit_l, perp_l = quantize(ctx, sd, "vq_model_l.", z_l)
    xh_l = decoder_forward(ctx, sd, "decoder_l.", zq_l, spec.dec_l, band_lf, spec.C, spec.T)
    z_h = encoder_forward(ctx, sd, "encoder_h.", x, spec.enc_h, band_hf)
    zq_h, s_h, commit_h, perp_h = quantize(ctx, sd, "vq_model_h.", z_h)
    xh_h = decoder_forward(ctx, sd, "decoder_h.", zq_h, spec.dec_h, band_hf, spec.C, spec.T)
    if return_x_rec:
        return xh_l + xh_h
    rl = F.mse_loss(x_l, xh_l)
    rh = F.l1_loss(x_h, xh_h)
    loss = rl + rh + commit_l + commit_h
    return dict(loss=loss, recons_lf=rl, recons_hf=rh, commit_lf=commit_l, commit_hf=commit_h,
                perp_lf=perp_l, perp_hf=perp_h, z_l=z_l, z_h=z_h, s_l=s_l, s_h=s_h,
                xhat_l=xh_l, xhat_h=xh_h)


def lr_at(step, base_lr, max_steps, warmup_rate=0.1, min_lr=1e-6):
    """Closed form of linear_warmup_cosine_annealingLR (utils/train_utils.py:451-483)."""
    warm = int(max_steps * warmup_rate)
    if step < warm:
        return base_lr * step / max(1, warm)
    t = step - warm
    T = max_steps - warm
    return min_lr + (base_lr - min_lr) * (1 + math.cos(math.pi * t / T)) / 2


# ----------------------------------------------------------------------------
# MaskGIT loops (models/maskgit.py) with injectable randomness
# ----------------------------------------------------------------------------
def gamma_cosine(r):
    """maskgit.py:218-228 ('cosine')."""
    return np.cos(r * np.pi / 2)


def random_mask_tokens(s, mask_token_id, ratio, rand):
    """_randomly_mask_tokens (maskgit.py:194-216) with the randomness injected.

    ratio: (b,) uniform[0,1) numpy; rand: (b,n) uniform torch.  mask=True keeps the token.
    Ties in `rand` resolve like torch.topk (larger first, then lower index).
    """
    b, n = s.shape
    n_unmask = np.clip(np.floor(gamma_cosine(ratio) * n), 0, n - 1).astype(int)
    mask = torch.zeros((b, n), dtype=torch.bool)
    for i in range(b):
        ind = rand[i].topk(int(n_unmask[i]), dim=-1).indices
        mask[i, ind] = True
    s_M = torch.where(mask, s, torch.full_like(s, mask_token_id))
    return s_M, mask


def race_sample(logits, s, mask_token_id, gumbel):
    """The categorical draw of first_pass/second_pass (maskgit.py:307-315) with injected noise.

    Categorical(logits).sample() runs torch.multinomial(probs, 1), whose n_sample = 1 path is
    the exponential race argmax_k p_k / q_k, q_k ~ Exp(1) (ATen Distributions.cpp,
    multinomial) -- in log form argmax_k l_k + g_k with Gumbel g_k = -log q_k.  The kernels
    add the injected fp32 g to the fp32 logits, so the keys here are the same fp32 sums and
    the argmax (first index of the maximum, as torch.argmax) is exact.  Known tokens are
    kept.  Also returns p(sampled) of the softmax in double (maskgit.py:320-326), +inf for
    known tokens."""
    keys = logits.float() + gumbel.float()
    sampled = keys.argmax(-1)
    unknown = s == mask_token_id
    sampled = torch.where(unknown, sampled, s)
    sel = torch.gather(F.softmax(logits.double(), dim=-1), -1, sampled.unsqueeze(-1)).squeeze(-1)
    sel = torch.where(unknown, sel, torch.full_like(sel, float("inf")))
    return sampled, sel


def remask_step(sel, sampled, mask_token_id, t, T, unknown0, temperature, u_gumbel):
    """mask_by_random_topk (maskgit.py:238-267, 317-346) on given p(sampled): confidence
    log(p + 1e-5) + temperature (1 - ratio) Gumbel(u_gumbel), the k = floor(unknown0 *
    gamma(ratio)) (float32, as the reference) lowest re-masked per row."""
    ratio = (t + 1) / T
    mask_ratio = gamma_cosine(ratio)
    mask_len = torch.clip(torch.floor(unknown0.float() * mask_ratio), min=0.0)
    g = -torch.log((-torch.log(u_gumbel.clamp(min=1e-20))).clamp(min=1e-20))
    conf = torch.log(sel.float() + 1e-5) + temperature * (1.0 - ratio) * g
    k = int(mask_len.unique().item())
    idx = torch.topk(conf, k=k, dim=-1, largest=False).indices
    masking = torch.zeros_like(conf, dtype=torch.bool)
    masking.scatter_(1, idx, True)
    return torch.where(masking, torch.full_like(sampled, mask_token_id), sampled)


def sample_step(logits, s, mask_token_id, t, T, unknown0, temperature, gumbel, u_gumbel):
    """One iteration of first_pass/second_pass (maskgit.py:302-346) with injected noise:
    race_sample, then remask_step on the fp32 softmax p(sampled) the reference gathers."""
    sampled, _ = race_sample(logits, s, mask_token_id, gumbel)
    unknown = s == mask_token_id
    sel = torch.gather(F.softmax(logits.float(), dim=-1), -1, sampled.unsqueeze(-1)).squeeze(-1)
    sel = torch.where(unknown, sel, torch.full_like(sel, float("inf")))
    return remask_step(sel, sampled, mask_token_id, t, T, unknown0, temperature, u_gumbel)


# ----------------------------------------------------------------------------
# Bidirectional transformer (bidirectional_transformer.py:34-251) with the
# x-transformers 1.3x encoder RESTATED (the package is absent: parity unpinned)
# ----------------------------------------------------------------------------
def xf_rmsnorm(x, g):
    """x-transformers RMSNorm: F.normalize(x, dim=-1) * sqrt(D) * g."""
    return F.normalize(x, dim=-1) * (x.shape[-1] ** 0.5) * g


def xf_blocks(sd, p, x, heads, depth, drop=0.0):
    """ContinuousTransformerWrapper(project_in, post_emb_norm, Encoder(pre_norm), project_out).
    drop > 0 (training): x-transformers' layer dropout (skip a branch with prob `drop`,
    host random() as the reference), attention-probability and FF dropout at `drop`."""
    import random
    h = F.linear(x, sd[p + "project_in.weight"])
    h = F.layer_norm(h, h.shape[-1:]) * sd[p + "post_emb_norm.gamma"]
    for i in range(2 * depth):
        if drop > 0 and random.random() < drop:
            continue
        q = f"{p}attn_layers.layers.{i}."
        n = xf_rmsnorm(h, sd[q + "0.0.g"])
        if i % 2 == 0:
            B, S, _ = n.shape
            qq = F.linear(n, sd[q + "1.to_q.weight"]).view(B, S, heads, 64).transpose(1, 2)
            kk = F.linear(n, sd[q + "1.to_k.weight"]).view(B, S, heads, 64).transpose(1, 2)
            vv = F.linear(n, sd[q + "1.to_v.weight"]).view(B, S, heads, 64).transpose(1, 2)
            att = torch.softmax(qq @ kk.transpose(-1, -2) * 64 ** -0.5, dim=-1)
            if drop > 0:
                att = F.dropout(att, drop)
            o = (att @ vv).transpose(1, 2).reshape(B, S, heads * 64)
            out = F.linear(o, sd[q + "1.to_out.weight"])
        else:
            u = F.gelu(F.linear(n, sd[q + "1.ff.0.0.weight"], sd[q + "1.ff.0.0.bias"]))
            if drop > 0:
                u = F.dropout(u, drop)
            out = F.linear(u, sd[q + "1.ff.2.weight"], sd[q + "1.ff.2.bias"])
        h = h + out
    h = xf_rmsnorm(h, sd[p + "attn_layers.final_norm.g"])
    return F.linear(h, sd[p + "project_out.weight"])


def upscale(ctx, sd, p, x, m):
    """Upscale (bidirectional_transformer.py:12-30): (b n d) -> (b m d)."""
    x = F.interpolate(x.transpose(1, 2), size=(m,), mode="nearest")
    x = F.conv1d(x, sd[p + "conv.0.weight"], sd[p + "conv.0.bias"], padding=1)
    x = F.gelu(x)
    x = _bn(ctx, sd, p + "conv.2.", x)
    x = F.conv1d(x, sd[p + "conv.3.weight"], sd[p + "conv.3.bias"], padding=1)
    return x.transpose(1, 2)


def transformer_forward(ctx, sd, kind, s_l, s_h, cls_idx, K, heads, depth, drop=0.0):
    """forward_lf / forward_hf (bidirectional_transformer.py:166-236); cls_idx (b,1) is the
    (already drop-resolved) class index (n_classes = uncond).  drop > 0: the reference's
    training-time dropouts at that rate (token-embedding dropout on non-mask tokens,
    :152-164, and the encoder's, xf_blocks) with torch's CPU RNG; 0: deterministic."""
    def tok_drop(s, e, mask_id):
        if drop <= 0:
            return e
        return torch.where((s == mask_id)[:, :, None], e, F.dropout(e, drop))
    tok = tok_drop(s_l, F.embedding(s_l, sd["tok_emb_l.weight"]), K)
    table = "tok_emb_l.weight"
    if kind == "hf":
        th = tok_drop(s_h, F.embedding(s_h, sd["tok_emb_h.weight"]), K)
        tok = torch.cat([upscale(ctx, sd, "projector.", tok, th.shape[1]), th], dim=-1)
        table = "tok_emb_h.weight"
    cls = F.embedding(cls_idx, sd["class_condition_emb.weight"])
    n = tok.shape[1]
    x = torch.cat([cls, tok + sd["pos_emb.weight"][:n]], dim=1)
    x = xf_blocks(sd, "blocks.", x, heads, depth, drop)
    x = F.linear(x, sd["pred_head.0.weight"], sd["pred_head.0.bias"])
    x = F.layer_norm(F.gelu(x), x.shape[-1:], sd["pred_head.2.weight"], sd["pred_head.2.bias"], 1e-12)
    x = x[:, 1:, :]
    logits = x @ sd[table].t() + sd["bias"]
    return logits[:, :, :-1]


def masked_ce(logits, s, keep):
    """maskgit.py:183-191."""
    return F.cross_entropy(logits[~keep].float(), s[~keep].long())


def _mask_by_random_topk_torch(mask_len, probs, temperature):
    """maskgit.py:238-267, same torch RNG consumption (uniform_ for the Gumbel noise)."""
    def log(t, eps=1e-20):
        return torch.log(t.clamp(min=eps))

    noise = torch.zeros_like(probs).uniform_(0, 1)
    confidence = torch.log(probs + 1e-5) + temperature * (-log(-log(noise)))
    k = int(mask_len.unique().item())
    ind = torch.topk(confidence, k=k, dim=-1, largest=False).indices
    masking = torch.zeros_like(confidence)
    masking.scatter_(1, ind, 1.0)
    return masking.bool()


def _pass_torch(logit_fn, s, mask_id, T, temp, unknown0):
    """first_pass / second_pass (maskgit.py:294-411) with torch's own sampling calls."""
    for t in range(T):
        logits = logit_fn(s)
        sampled = torch.distributions.categorical.Categorical(logits=logits).sample()
        unknown = s == mask_id
        sampled = torch.where(unknown, sampled, s)
        ratio = 1.0 * (t + 1) / T
        mask_ratio = gamma_cosine(ratio)
        probs = F.softmax(logits, dim=-1)
        sel = torch.gather(probs, dim=-1, index=sampled.unsqueeze(-1)).squeeze()
        sel = torch.where(unknown, sel, torch.Tensor([torch.inf]))
        mask_len = torch.clip(torch.unsqueeze(torch.floor(unknown0 * mask_ratio), 1), min=0.0)
        masking = _mask_by_random_topk_torch(mask_len, sel, temp * (1.0 - ratio))
        s = torch.where(masking, mask_id, sampled)
    return s


def iterative_decoding_torch(tf_l, tf_h, num, n_l, n_h, mask_l, mask_h, T, temp_l, temp_h):
    """iterative_decoding (maskgit.py:413-446), unconditional, CPU, torch RNG."""
    s_l = (mask_l * torch.ones((num, n_l))).to(torch.int64)
    s_h = (mask_h * torch.ones((num, n_h))).to(torch.int64)
    unk_l = torch.sum(s_l == mask_l, dim=-1)
    unk_h = torch.sum(s_h == mask_h, dim=-1)
    s_l = _pass_torch(tf_l, s_l, mask_l, T["lf"], temp_l, unk_l)
    s_h = _pass_torch(lambda sh: tf_h(s_l, sh), s_h, mask_h, T["hf"], temp_h, unk_h)
    return s_l, s_h


# ----------------------------------------------------------------------------
# FidelityEnhancer / Unet1D forward (models/fidelity_enhancer.py), eval mode
# ----------------------------------------------------------------------------
def fe_ws_conv(x, w, b, stride=1, padding=0):
    """WeightStandardizedConv2d.forward (fidelity_enhancer.py:96-116): per output channel,
    (w - mean) * rsqrt(var_biased + 1e-5), then conv1d."""
    mean = w.mean(dim=(1, 2), keepdim=True)
    var = w.var(dim=(1, 2), unbiased=False, keepdim=True)
    return F.conv1d(x, (w - mean) * (var + 1e-5).rsqrt(), b, stride, padding)


def fe_layernorm(x, g):
    """LayerNorm over the channel axis, gamma only (fidelity_enhancer.py:119-127)."""
    var = torch.var(x, dim=1, unbiased=False, keepdim=True)
    mean = torch.mean(x, dim=1, keepdim=True)
    return (x - mean) * (var + 1e-5).rsqrt() * g


def fe_block(sd, p, x, groups):
    """Block.forward (fidelity_enhancer.py:182-204): WS conv3 -> GroupNorm -> Snake ->
    Dropout (identity in eval); scale_shift is never passed (Unet1D.forward :402-405)."""
    x = fe_ws_conv(x, sd[p + "proj.weight"], sd[p + "proj.bias"], padding=1)
    x = F.group_norm(x, groups, sd[p + "norm.weight"], sd[p + "norm.bias"], 1e-5)
    a = sd[p + "act.a"]
    return x + (1 / a) * torch.sin(a * x) ** 2


def fe_resnet(sd, p, x, groups):
    """ResnetBlock.forward (fidelity_enhancer.py:219-231) without a time embedding."""
    h = fe_block(sd, p + "block1.", x, groups)
    h = fe_block(sd, p + "block2.", h, groups)
    res = F.conv1d(x, sd[p + "res_conv.weight"], sd[p + "res_conv.bias"]) \
        if p + "res_conv.weight" in sd else x
    return h + res


def fe_linear_attention(sd, p, x, heads=4, dim_head=32):
    """Residual(PreNorm(LinearAttention)) (fidelity_enhancer.py:75-82,130-137,234-260)."""
    b, c, n = x.shape
    xn = fe_layernorm(x, sd[p + "norm.g"])
    q, k, v = F.conv1d(xn, sd[p + "fn.to_qkv.weight"]).chunk(3, dim=1)
    q, k, v = (t.reshape(b, heads, dim_head, n) for t in (q, k, v))
    q = q.softmax(dim=-2) * dim_head ** -0.5
    k = k.softmax(dim=-1)
    context = torch.einsum("bhdn,bhen->bhde", k, v)
    out = torch.einsum("bhde,bhdn->bhen", context, q).reshape(b, heads * dim_head, n)
    out = F.conv1d(out, sd[p + "fn.to_out.0.weight"], sd[p + "fn.to_out.0.bias"])
    return fe_layernorm(out, sd[p + "fn.to_out.1.g"]) + x


def fe_attention(sd, p, x, heads=4, dim_head=32):
    """Residual(PreNorm(Attention)) (fidelity_enhancer.py:263-283)."""
    b, c, n = x.shape
    xn = fe_layernorm(x, sd[p + "norm.g"])
    q, k, v = F.conv1d(xn, sd[p + "fn.to_qkv.weight"]).chunk(3, dim=1)
    q, k, v = (t.reshape(b, heads, dim_head, n) for t in (q, k, v))
    attn = torch.einsum("bhdi,bhdj->bhij", q * dim_head ** -0.5, k).softmax(dim=-1)
    out = torch.einsum("bhij,bhdj->bhid", attn, v)
    out = out.permute(0, 1, 3, 2).reshape(b, heads * dim_head, n)
    return F.conv1d(out, sd[p + "fn.to_out.weight"], sd[p + "fn.to_out.bias"]) + x


def _fe_upsample(sd, p, x):
    """Upsample (fidelity_enhancer.py:85-89): nearest x2 then conv3 p1."""
    x = F.interpolate(x, scale_factor=2, mode="nearest")
    return F.conv1d(x, sd[p + "1.weight"], sd[p + "1.bias"], padding=1)


def fe_forward(sd, x_a, input_length, dim_mults=(1, 2, 4, 8), groups=4):
    """FidelityEnhancer.forward (fidelity_enhancer.py:484-498) -> Unet1D.forward
    (:395-455).  `sd` holds the FidelityEnhancer state_dict (keys `unet.*`)."""
    sd = {k[5:]: v for k, v in sd.items() if k.startswith("unet.")}
    x = F.interpolate(x_a, size=input_length, mode="linear", align_corners=False)
    x = F.conv1d(x, sd["init_conv.weight"], sd["init_conv.bias"], padding=3)
    r = x.clone()
    h = []
    n = len(dim_mults)
    for i in range(n):
        p = f"downs.{i}."
        x = fe_resnet(sd, p + "0.", x, groups)
        h.append(x)
        x = fe_resnet(sd, p + "1.", x, groups)
        x = fe_linear_attention(sd, p + "2.fn.", x)
        h.append(x)
        if i < n - 1:  # Downsample: conv k4 s2 p1 (:92-93)
            x = F.conv1d(x, sd[p + "3.weight"], sd[p + "3.bias"], stride=2, padding=1)
        else:
            x = F.conv1d(x, sd[p + "3.weight"], sd[p + "3.bias"], padding=1)
    x = fe_resnet(sd, "mid_block1.", x, groups)
    x = fe_attention(sd, "mid_attn.fn.", x)
    x = fe_resnet(sd, "mid_block2.", x, groups)
    for i in range(n):
        p = f"ups.{i}."
        hh = F.interpolate(h.pop(), size=x.shape[-1], mode="linear", align_corners=False)
        x = fe_resnet(sd, p + "0.", torch.cat((x, hh), dim=1), groups)
        hh = F.interpolate(h.pop(), size=x.shape[-1], mode="linear", align_corners=False)
        x = fe_resnet(sd, p + "1.", torch.cat((x, hh), dim=1), groups)
        x = fe_linear_attention(sd, p + "2.fn.", x)
        if i < n - 1:
            x = _fe_upsample(sd, p + "3.", x)
        else:
            x = F.conv1d(x, sd[p + "3.weight"], sd[p + "3.bias"], padding=1)
    x = _fe_upsample(sd, "last_up.", x)
    x = F.interpolate(x, size=r.shape[-1], mode="linear", align_corners=False)
    x = fe_resnet(sd, "final_res_block.", torch.cat((x, r), dim=1), groups)
    x = F.conv1d(x, sd["final_conv.0.weight"], sd["final_conv.0.bias"])
    for j in (1, 2):  # conv3, replicate padding (:386-392)
        x = F.conv1d(F.pad(x, (1, 1), mode="replicate"), sd[f"final_conv.{j}.weight"],
                     sd[f"final_conv.{j}.bias"])
    return x


# ----------------------------------------------------------------------------
# FID (evaluation/eval_utils.py:56-81)
# ----------------------------------------------------------------------------
def fid_moments(z):
    """z.mean(0) (in z's dtype, as numpy does) and np.cov(z, rowvar=False) (float64)."""
    return z.mean(axis=0), np.cov(z, rowvar=False)


def fid(z1, z2):
    """calculate_fid: |mu1 - mu2|^2 + tr(s1 + s2 - 2 sqrtm(s1 s2)), real part of sqrtm."""
    from scipy.linalg import sqrtm
    mu1, s1 = fid_moments(z1)
    mu2, s2 = fid_moments(z2)
    cm = sqrtm(s1.dot(s2))
    if np.iscomplexobj(cm):
        cm = cm.real
    return ((mu1 - mu2) ** 2.0).sum() + np.trace(s1 + s2 - 2.0 * cm)
