"""TEST INFRASTRUCTURE / CPU BASELINE ONLY — the reference's stage1+stage2 train step
restated on torch CPU (the `cpu_baseline` leg of bench.py; "port" kind).

Same work as one product joint step: stage1 forward/backward/AdamW
(trainers/stage1.py:89-236) then stage2 forward/backward/AdamW with the frozen
stage1 encoders (trainers/stage2.py:49-68, models/maskgit.py:155-216), dropouts as
in the reference: ResBlock 0.3; in the priors token-embedding, attention, FF and layer
dropout 0.3 and the classifier-free-guidance class drop 0.2
(configs/config.yaml:48-64).  tools/cpu_ref_compare.py times its stage1 / stage2 halves
against the reference's own files in the build container (DESIGN.md §CPU baseline).
"""
import time

import numpy as np
import torch
import torch.nn.functional as F

from . import tvq_oracle as O


def _init_stage1(spec, K, hid, seed=0):
    """Deterministic random weights shaped like trainers/stage1.py's module tree."""
    g = torch.Generator().manual_seed(seed)
    sd = {}

    def conv(p, co, ci, kh, kw, t=False):
        shape = (ci, co, kh, kw) if t else (co, ci, kh, kw)
        sd[p + "weight"] = torch.randn(shape, generator=g) / np.sqrt(ci * kh * kw)
        sd[p + "bias"] = torch.zeros(co)

    def bn(p, c):
        sd[p + "weight"] = torch.ones(c)
        sd[p + "bias"] = torch.zeros(c)
        sd[p + "running_mean"] = torch.zeros(c)
        sd[p + "running_var"] = torch.ones(c)
        sd[p + "num_batches_tracked"] = torch.tensor(0)

    def snake(p, c):
        sd[p + "a"] = torch.rand(1, c, 1, 1, generator=g) * 0.3 + 0.2

    for br, enc, dec in (("l", spec.enc_l, spec.dec_l), ("h", spec.enc_h, spec.dec_h)):
        for i, (kind, ci, co) in enumerate(enc):
            p = f"encoder_{br}.encoder.{i}."
            if kind == "enc":
                conv(p + "block.0.", co, ci, 3, 4); bn(p + "block.1.", co); snake(p + "block.2.", co)
            else:
                _res(sd, p, ci, co, conv, bn, snake)
        for i, (kind, ci, co) in enumerate(dec):
            p = f"decoder_{br}.decoder.{i}."
            if kind == "res":
                _res(sd, p, ci, co, conv, bn, snake)
            elif kind == "dec":
                conv(p + "block.0.", co, ci, 3, 4, t=True); bn(p + "block.1.", co); snake(p + "block.2.", co)
            else:
                conv(p, co, ci, 3, 4, t=True)
        sd[f"decoder_{br}.linear.weight"] = torch.randn(spec.T, spec.T, generator=g) / np.sqrt(spec.T)
        sd[f"decoder_{br}.linear.bias"] = torch.zeros(spec.T)
        E = torch.randn(K, hid, generator=g)
        sd[f"vq_model_{br}._codebook.embed"] = E
        sd[f"vq_model_{br}._codebook.embed_avg"] = E.clone()
        sd[f"vq_model_{br}._codebook.cluster_size"] = torch.zeros(K)
    return sd


def _res(sd, p, ci, co, conv, bn, snake):
    snake(p + "convs.0.", ci)
    conv(p + "convs.1.", co, ci, 3, 3)
    bn(p + "convs.2.", co)
    snake(p + "convs.3.", co)
    conv(p + "convs.4.", co, co, 3, 3)
    if ci != co:
        conv(p + "proj.", co, ci, 1, 1)


def _init_xf(kind, K, emb, hidden, depth, heads, ntok, n_classes, seed):
    g = torch.Generator().manual_seed(seed)
    in_dim = emb if kind == "lf" else 2 * emb
    r = lambda *s: torch.randn(*s, generator=g) * 0.02
    sd = {"tok_emb_l.weight": r(K + 1, emb), "pos_emb.weight": r(ntok + 1, in_dim),
          "class_condition_emb.weight": r(n_classes + 1, in_dim),
          "blocks.project_in.weight": r(hidden, in_dim), "blocks.post_emb_norm.gamma": torch.ones(hidden),
          "blocks.project_out.weight": r(in_dim, hidden),
          "blocks.attn_layers.final_norm.g": torch.ones(hidden),
          "pred_head.0.weight": r(emb, in_dim), "pred_head.0.bias": torch.zeros(emb),
          "pred_head.2.weight": torch.ones(emb), "pred_head.2.bias": torch.zeros(emb),
          "bias": torch.zeros(ntok, K + 1)}
    if kind == "hf":
        sd["tok_emb_h.weight"] = r(K + 1, emb)
        sd["projector.conv.0.weight"] = r(2 * emb, emb, 3); sd["projector.conv.0.bias"] = torch.zeros(2 * emb)
        sd["projector.conv.2.weight"] = torch.ones(2 * emb); sd["projector.conv.2.bias"] = torch.zeros(2 * emb)
        sd["projector.conv.2.running_mean"] = torch.zeros(2 * emb)
        sd["projector.conv.2.running_var"] = torch.ones(2 * emb)
        sd["projector.conv.2.num_batches_tracked"] = torch.tensor(0)
        sd["projector.conv.3.weight"] = r(emb, 2 * emb, 3); sd["projector.conv.3.bias"] = torch.zeros(emb)
    for i in range(2 * depth):
        p = f"blocks.attn_layers.layers.{i}."
        sd[p + "0.0.g"] = torch.ones(hidden)
        if i % 2 == 0:
            for w in ("to_q", "to_k", "to_v"):
                sd[p + f"1.{w}.weight"] = r(heads * 64, hidden)
            sd[p + "1.to_out.weight"] = r(hidden, heads * 64)
        else:
            sd[p + "1.ff.0.0.weight"] = r(hidden, hidden); sd[p + "1.ff.0.0.bias"] = torch.zeros(hidden)
            sd[p + "1.ff.2.weight"] = r(hidden, hidden); sd[p + "1.ff.2.bias"] = torch.zeros(hidden)
    return sd


class JointStep:
    """One stage1 + one stage2 optimizer step of the reference, on torch CPU."""

    def __init__(self, B=256, C=6, T=256, K=512, hid=128, n_classes=5, seed=0):
        self.spec = O.Stage1Spec(T, C, 4, hid)
        self.K = K
        sd = _init_stage1(self.spec, K, hid, seed)
        self.s1_params = {k: v.requires_grad_(True) for k, v in sd.items()
                          if v.is_floating_point() and not k.split(".")[-1] in
                          ("running_mean", "running_var", "embed", "embed_avg", "cluster_size")}
        self.sd1 = sd
        self.opt1 = torch.optim.AdamW(list(self.s1_params.values()), lr=1e-3)
        self.frozen = {k: v.detach().clone() for k, v in sd.items()}
        self.xl = _init_xf("lf", K, hid, 128, 4, 2, 24, n_classes, seed + 1)
        self.xh = _init_xf("hf", K, hid, 32, 1, 1, 96, n_classes, seed + 2)
        self.xf_params = [v.requires_grad_(True) for d in (self.xl, self.xh) for k, v in d.items()
                          if v.is_floating_point() and "running" not in k]
        self.opt2 = torch.optim.AdamW(self.xf_params, lr=1e-3)
        g = torch.Generator().manual_seed(1234)
        x = torch.cumsum(0.1 * torch.randn(B, C, T, generator=g), -1)
        self.x = 2 * (x - x.amin(0, keepdim=True)) / (x.amax(0, keepdim=True) - x.amin(0, keepdim=True) + 1e-8) - 1
        self.y = torch.randint(0, n_classes, (B, 1), generator=g)
        self.rng = np.random.default_rng(0)

    def step(self):
        return self.step_stage1(), self.step_stage2()

    def step_stage1(self):
        self.opt1.zero_grad()
        ctx = O.Ctx(True, dropout_p=0.3)
        out = O.stage1_forward(ctx, self.sd1, self.spec, self.x)
        out["loss"].backward()
        self.opt1.step()
        with torch.no_grad():
            for k, v in ctx.updates.items():
                self.sd1[k] = v.detach()
        return float(out["loss"].detach())

    def step_stage2(self, drop=0.3, p_uncond=0.2):
        """frozen stage1 snapshot (eval) -> tokens -> masking -> priors -> masked CE."""
        self.opt2.zero_grad()
        with torch.no_grad():
            e = O.Ctx(False)
            z_l = O.encoder_forward(e, self.frozen, "encoder_l.", self.x, self.spec.enc_l, O.band_lf)
            _, s_l, _, _ = O.quantize(e, self.frozen, "vq_model_l.", z_l)
            z_h = O.encoder_forward(e, self.frozen, "encoder_h.", self.x, self.spec.enc_h, O.band_hf)
            _, s_h, _, _ = O.quantize(e, self.frozen, "vq_model_h.", z_h)
        B = s_l.shape[0]
        sMl, kl = O.random_mask_tokens(s_l, self.K, self.rng.uniform(0, 1, B), torch.rand(s_l.shape))
        sMh, kh = O.random_mask_tokens(s_h, self.K, self.rng.uniform(0, 1, B), torch.rand(s_h.shape))
        c = O.Ctx(True)
        uncond = torch.full_like(self.y, 5)
        ll = O.transformer_forward(c, self.xl, "lf", sMl, None,
                                   torch.where(torch.rand(self.y.shape) > p_uncond, self.y, uncond),
                                   self.K, 2, 4, drop=drop)
        lh = O.transformer_forward(c, self.xh, "hf", sMl, sMh,
                                   torch.where(torch.rand(self.y.shape) > p_uncond, self.y, uncond),
                                   self.K, 1, 1, drop=drop)
        loss = O.masked_ce(ll, s_l, kl) + O.masked_ce(lh, s_h, kh)
        loss.backward()
        self.opt2.step()
        return float(loss.detach())


def cpu_model():
    """The host CPU's model string (/proc/cpuinfo), for the bench's cpu_baseline record."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def _median_step(fn, steps, warmup):
    """BASELINE.md §3 protocol: `warmup` untimed steps, then the median of `steps` timed
    steps (each timed alone).  Returns (median seconds, every step's seconds)."""
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


def measure(threads, steps=5, warmup=2, B=256, detail=False):
    """Seconds per joint step of the CPU restatement: median of `steps` (>= 5) timed steps
    after `warmup` (2) untimed ones."""
    torch.set_num_threads(threads)
    js = JointStep(B=B)
    med, ts = _median_step(js.step, steps, warmup)
    return (med, ts) if detail else med


def measure_stage1(threads, B, T, K, steps=5, warmup=2):
    """Seconds per stage1 train step (BASELINE configs[0]: T=128, K=256, config.yaml
    widths) of the CPU restatement: median of `steps` after `warmup`."""
    torch.set_num_threads(threads)
    js = JointStep(B=B, T=T, K=K)
    return _median_step(js.step_stage1, steps, warmup)[0]


def sampler_fn(num=256, seed=0, K=512, hid=128, n_classes=5, T=256, C=6):
    """One batch of `num` unconditional samples of the CPU restatement as a callable:
    iterative_decoding (maskgit.py:413-446: 10 LF + 1 HF steps, torch sampling) +
    decode_token_ind_to_timeseries for LF and HF (maskgit.py:448-477) -- the work of
    generation/sampler.py per batch."""
    spec = O.Stage1Spec(T, C, 4, hid)
    sd = _init_stage1(spec, K, hid, seed)
    xl = _init_xf("lf", K, hid, 128, 4, 2, 24, n_classes, seed + 1)
    xh = _init_xf("hf", K, hid, 32, 1, 1, 96, n_classes, seed + 2)
    e = O.Ctx(False)
    uncond = lambda b: torch.full((b, 1), n_classes, dtype=torch.int64)  # noqa: E731
    tf_l = lambda s: O.transformer_forward(e, xl, "lf", s, None, uncond(s.shape[0]), K, 2, 4)  # noqa: E731
    tf_h = lambda sl, sh: O.transformer_forward(e, xh, "hf", sl, sh, uncond(sl.shape[0]), K, 1, 1)  # noqa: E731

    def run():
        with torch.no_grad():
            s_l, s_h = O.iterative_decoding_torch(tf_l, tf_h, num, 24, 96, K, K, {"lf": 10, "hf": 1},
                                                  10, 4)
            out = 0
            for br, s, plan, band, W in (("l", s_l, spec.dec_l, O.band_lf, 8),
                                         ("h", s_h, spec.dec_h, O.band_hf, 32)):
                z = F.embedding(s, sd[f"vq_model_{br}._codebook.embed"])
                z = z.transpose(1, 2).reshape(num, hid, 3, W)
                out = out + O.decoder_forward(e, sd, f"decoder_{br}.", z, plan, band, C, T)
            return out
    return run


def measure_sampler(threads, num=256, reps=1, seed=0, **kw):
    """Seconds per `num` unconditional samples of the CPU restatement (sampler_fn)."""
    torch.set_num_threads(threads)
    run = sampler_fn(num, seed, **kw)
    run()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    return (time.perf_counter() - t0) / reps
