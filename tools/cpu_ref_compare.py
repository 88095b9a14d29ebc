"""Validate the CPU baseline port (oracle/cpu_baseline.py) against the reference's own CPU
step, timed side by side in the BUILD CONTAINER at equal thread counts (SURVEY §8(d)
step 3 asks for agreement within +-10 %).  Reads /root/reference (absent on the GPU box);
the reference files are loaded by file path exactly as tests/golden/make_golden.py does
(stage2: with its x-transformers stub, the T1 restatement).

usage: python tools/cpu_ref_compare.py [threads] > profiles/r02_cpu_ref_compare.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import make_golden as MG  # noqa: E402
from oracle import cpu_baseline  # noqa: E402

PRIOR = {"p_unconditional": 0.2, "model_dropout": 0.3, "emb_dropout": 0.3}


def batch(B, C, T, seed=1234):
    g = torch.Generator().manual_seed(seed)
    x = torch.cumsum(0.1 * torch.randn(B, C, T, generator=g), -1)
    x = 2 * (x - x.amin(0, keepdim=True)) / (x.amax(0, keepdim=True) - x.amin(0, keepdim=True) + 1e-8) - 1
    return x, torch.randint(0, 5, (B, 1), generator=g)


def interleaved(fa, fb, steps, warmup=2):
    """Median seconds per step of fa and of fb, timed alternately step by step (after
    `warmup` untimed steps of each), so drift of the shared host hits both alike."""
    for _ in range(warmup):
        fa()
        fb()
    ta, tb = [], []
    for _ in range(steps):
        t0 = time.perf_counter()
        fa()
        ta.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        fb()
        tb.append(time.perf_counter() - t0)
    return float(np.median(ta)), float(np.median(tb))


def ref_stage1(ref, B, T, K):
    torch.manual_seed(0)
    np.random.seed(0)
    cfg = MG._stage1_config(4, 128, K)
    m = ref.stage1.Stage1(T, 6, cfg).train()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    x, y = batch(B, 6, T)

    def step():
        opt.zero_grad(set_to_none=True)
        recons, vq, _ = m((x, y), 0)
        loss = recons["LF.time"] + recons["HF.time"] + vq["LF"]["loss"] + vq["HF"]["loss"]
        loss.sum().backward()
        opt.step()
    return step


def ref_stage2(ref, bt, maskgit, B, T, K):
    """MaskGIT.forward (reference file) over a frozen reference stage1, AdamW over the
    priors (trainers/stage2.py:49-68,112-119)."""
    torch.manual_seed(0)
    np.random.seed(0)
    cfg = MG._stage1_config(4, 128, K)
    s1 = ref.stage1.Stage1(T, 6, cfg)
    x, y = batch(B, 6, T)
    s1.eval()
    with torch.no_grad():
        s1.encoder_l(x), s1.encoder_h(x)
    mgc = maskgit.MaskGIT
    mg = mgc.__new__(mgc)
    nn.Module.__init__(mg)
    mg.choice_temperature_l, mg.choice_temperature_h = 10, 4
    mg.T, mg.n_classes, mg.cfg_scale = {"lf": 10, "hf": 1}, 5, 1.0
    mg.mask_token_ids = {"lf": K, "hf": K}
    mg.gamma = mg.gamma_func("cosine")
    mg.stage1 = s1
    for n in ("encoder_l", "decoder_l", "vq_model_l", "encoder_h", "decoder_h", "vq_model_h"):
        setattr(mg, n, getattr(s1, n))
    nl, nh = int(s1.encoder_l.num_tokens), int(s1.encoder_h.num_tokens)
    mg.num_tokens_l, mg.num_tokens_h = nl, nh
    mg.transformer_l = bt.BidirectionalTransformer("lf", nl, {"lf": K, "hf": K}, 128, n_classes=5,
                                                   **MG.PRIOR_L, **PRIOR)
    mg.transformer_h = bt.BidirectionalTransformer("hf", nh, {"lf": K, "hf": K}, 128, n_classes=5,
                                                   num_tokens_l=nl, **MG.PRIOR_H, **PRIOR)
    for p in s1.parameters():
        p.requires_grad_(False)
    mg.train()
    params = [p for p in mg.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=1e-3)

    def step():
        opt.zero_grad(set_to_none=True)
        loss, _ = mg(x, y)
        loss.backward()
        opt.step()
    return step


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.set_num_threads(threads)
    ref = MG.load_reference()
    bt, maskgit = MG.load_reference_stage2(ref)
    from oracle.cpu_baseline import cpu_model
    res = {"threads": threads, "cpu": cpu_model(),
           "protocol": "reference and port steps alternated; 2 untimed warmups each, then the "
                       "median of 7 timed steps each", "rows": []}
    for name, B, T, K in (("stage1 configs[1] (B=256,T=256,K=512)", 256, 256, 512),
                          ("stage1 configs[0] (B=32,T=128,K=256)", 32, 128, 256),
                          ("stage1 configs[0] (B=256,T=128,K=256)", 256, 128, 256)):
        js = cpu_baseline.JointStep(B=B, T=T, K=K)
        r, p = interleaved(ref_stage1(ref, B, T, K), js.step_stage1, 7)
        res["rows"].append({"what": name, "reference_s": round(r, 4), "port_s": round(p, 4),
                            "port_over_reference": round(p / r, 3)})
        print(json.dumps(res["rows"][-1]), file=sys.stderr, flush=True)
    js = cpu_baseline.JointStep(B=256)
    r, p = interleaved(ref_stage2(ref, bt, maskgit, 256, 256, 512), js.step_stage2, 7)
    res["rows"].append({"what": "stage2 configs[2] (B=256,T=256,K=512; T1 restated in both)",
                        "reference_s": round(r, 4), "port_s": round(p, 4),
                        "port_over_reference": round(p / r, 3)})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
