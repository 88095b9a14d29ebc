"""Isolated timings of the fused prior / ResBlock kernels at the bench's shapes (graph-replayed
launches timed with HIP events on their stream, as bench.py's roofline legs):
  attn_fwd / attn_bwd   tvq_attn_branch_fwd / _bwd, 256 sequences x 25 tokens (the LF prior)
  ffn_fwd / ffn_bwd     tvq_ffn_fwd / _bwd, 6400 rows
  rb64_fwd / rb64_bwd   the C = 64 fused ResBlock on (256, 64, 3, 8) (fwd: 2 kernels + the
                        BN finish; bwd: 2 kernels + finish + 2 weight gradients + slab sum)
usage: python tools/fused_bench.py [reps]"""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import _graph_time_us  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    from timevqvae.hip import rng
    from timevqvae.hip._native import call, ptr, stream_ptr, value
    dev = torch.device("cuda", 0)
    rng.manual_seed(1)
    out = {}
    B, S, D = 256, 25, 128
    M = B * S
    g = torch.Generator(device="cpu").manual_seed(3)
    rnd = lambda *sh, s=1.0: (torch.randn(*sh, generator=g) * s).to(dev)  # noqa: E731
    x, gy = rnd(M, D), rnd(M, D)
    W, Wo, gn = rnd(3 * D, D, s=0.08), rnd(D, D, s=0.08), 1 + rnd(D, s=0.1)
    gate = torch.ones(1, device=dev)
    seed = rng.seed_tensor(dev)
    y, xn, o, dx, gg = (torch.empty(M, D, device=dev) for _ in range(5))
    inv = torch.empty(M, device=dev)
    qkv, dqkv = torch.empty(M, 3 * D, device=dev), torch.empty(M, 3 * D, device=dev)
    lse = torch.empty(B * 2 * S, device=dev)
    dg = torch.zeros(D, device=dev)
    ws = torch.empty(value("tvq_attn_branch_workspace", B, D), device=dev)
    fwd = (lambda: call("tvq_attn_branch_fwd", ptr(x), B, S, D, 2, ptr(gn), math.sqrt(D), ptr(W),
                        ptr(Wo), ptr(gate), 0.3, ptr(seed), 0, ptr(y), ptr(xn), ptr(inv), ptr(qkv),
                        ptr(o), ptr(lse), stream_ptr()))
    bwd = (lambda: call("tvq_attn_branch_bwd", ptr(gy), ptr(x), B, S, D, 2, ptr(gn), math.sqrt(D),
                        ptr(inv), ptr(W), ptr(Wo), ptr(gate), 0.3, ptr(seed), 0, ptr(qkv), ptr(o),
                        ptr(lse), ptr(dx), ptr(dqkv), ptr(gg), ptr(dg), 0, ptr(ws), stream_ptr()))
    with torch.no_grad():
        out["attn_fwd_us"] = round(_graph_time_us([fwd], reps), 2)
        out["attn_bwd_us"] = round(_graph_time_us([bwd], reps), 2)
        W1, W2, b1, b2 = rnd(D, D, s=0.08), rnd(D, D, s=0.08), rnd(D, s=0.1), rnd(D, s=0.1)
        pre, hd, dpre, dxn = (torch.empty(M, D, device=dev) for _ in range(4))
        ffw = (lambda: call("tvq_ffn_fwd", ptr(x), ptr(gy), M, D, ptr(W1), ptr(b1), ptr(W2), ptr(b2),
                            ptr(gate), 0.3, ptr(seed), 0, ptr(y), ptr(pre), ptr(hd), stream_ptr()))
        ffb = (lambda: call("tvq_ffn_bwd", ptr(gy), ptr(pre), M, D, ptr(W1), ptr(W2), ptr(gate), 0.3,
                            ptr(seed), 0, ptr(dpre), ptr(dxn), ptr(gg), stream_ptr()))
        out["ffn_fwd_us"] = round(_graph_time_us([ffw], reps), 2)
        out["ffn_bwd_us"] = round(_graph_time_us([ffb], reps), 2)
    out["mfma_floor_us"] = {"attn_fwd": round(288 * 64 / 2.1e3, 2), "attn_bwd": round(336 * 64 / 2.1e3, 2),
                            "ffn": round(128 * 64 / 2.1e3, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
