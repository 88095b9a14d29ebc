"""Algorithmic FLOPs of one joint train step, counted with torch.utils.flop_counter over the
CPU restatement of the same module tree (oracle/cpu_baseline.JointStep: config.yaml
architecture, K=512, T=256, C=6), at a small batch and scaled per trajectory.

Counted: every conv / matmul / bmm / addmm of stage1 forward+backward and of stage2 (frozen
encoders forward, both priors forward+backward); not counted: FFTs, norms, elementwise work and
the optimizer.  The VQ distance matmul (2*K*hid per token) is counted; the restatement's
one-hot EMA matmul (vq.py:229's embed_sum as onehot.T @ x) is subtracted, since the EMA is a
segmented sum, not a GEMM.  Stage2 is counted
with layer dropout off (every branch run: the upper bound of the per-step work).

The sampler batch (BASELINE configs[4]: iterative decoding of 10 LF + 1 HF steps with the
priors' forwards, then both decoders) is counted the same way, per 1024 trajectories.

`sampler_executed_gflop_per_1024` is what the HIP sampler executes: the same count less the
Linears its eval heads compose away (hip path, models/bidirectional_transformer.py
_head_hf_eval and the LF prior's folded tables), from the config.yaml shapes:
  LF project_in (128 -> 128) on 25 tokens x 10 decoding steps, folded into the tables, and
  LF project_out (128 -> 128) composed with pred_head's Linear (one 128 -> 128 Linear);
  HF Upscale's last conv 256 -> 128 (k 3) becomes 256 -> 32 (project_in's tl half folded in);
  HF project_in (256 -> 32) on 97 tokens: its th half gathered from a projected table;
  HF project_out (32 -> 256) then pred_head's Linear (256 -> 128): one 32 -> 128 Linear.
(the folded tables themselves, once per batch, are < 0.05 GFLOP and not subtracted)
`step_executed_gflop_at_B256`: the train step less what the priors' training forwards fold
(Upscale's last conv with the HF project_in's tl half; project_out with pred_head's Linear in
both priors; the weight products themselves, < 0.02 GFLOP per step, not subtracted).

usage: python tools/count_step_flops.py [B] > profiles/r05_step_flops.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.utils.flop_counter import FlopCounterMode  # noqa: E402

from oracle import cpu_baseline  # noqa: E402


def count(fn):
    with FlopCounterMode(display=False) as fc:
        fn()
    return fc.get_total_flops(), {str(k): v for k, v in fc.get_flop_counts()["Global"].items()}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.manual_seed(0)
    js = cpu_baseline.JointStep(B=B)
    f1, by1 = count(js.step_stage1)
    f2, by2 = count(lambda: js.step_stage2(drop=0.0))
    K, hid = 512, 128
    tokens = B * (3 * 8 + 3 * 32)  # LF 3x8 and HF 3x32 token grids
    f1 -= 2 * hid * tokens * K  # one-hot EMA matmul of the restatement (stage1 only)
    # sampler (BASELINE configs[4]): one batch = 10 LF + 1 HF prior forwards + both decoders
    fs, bys = count(cpu_baseline.sampler_fn(num=B))
    n_l, n_h, d_l, D_h, d_h, H_up, steps_l = 24, 96, 128, 128, 32, 256, 10
    saved = (2 * 2 * d_l * d_l * (n_l + 1) * steps_l  # LF project_in; project_out composed
             + 2 * n_h * H_up * 3 * (D_h - d_h)  # Upscale last conv 256 -> 128 vs -> 32
             + 2 * (n_h + 1) * 2 * D_h * d_h  # HF project_in
             + 2 * n_h * (d_h * 2 * D_h + 2 * D_h * D_h - d_h * D_h))  # project_out + pred_head
    # the train step (B = 256): what the priors' folded training forwards skip, each Linear /
    # conv counted 3x (forward, input gradient, weight gradient)
    L_l = 128
    step_saved = 3 * (2 * n_h * H_up * 3 * (D_h - d_h)  # Upscale last conv -> 32 channels
                      + 2 * (n_h + 1) * 2 * D_h * d_h - 2 * n_h * D_h * d_h  # HF project_in
                      + 2 * (n_h + 1) * d_h * 2 * D_h + 2 * n_h * 2 * D_h * D_h
                      - 2 * n_h * d_h * D_h  # HF project_out + pred_head -> one 32 -> 128
                      + 2 * (n_l + 1) * L_l * L_l)  # LF project_out folded into pred_head
    out = {"batch_counted": B,
           "step_executed_gflop_at_B256": ((f1 + f2) / B - step_saved) * 256 / 1e9,
           "sampler_gflop_per_1024": fs / B * 1024 / 1e9, "sampler_by_op": bys,
           "sampler_executed_gflop_per_1024": fs / B * 1024 / 1e9 - saved * 1024 / 1e9,
           "stage1_gflop_per_traj": f1 / B / 1e9, "stage2_gflop_per_traj": f2 / B / 1e9,
           "step_gflop_at_B256": (f1 + f2) / B * 256 / 1e9,
           "stage1_by_op": by1, "stage2_by_op": by2}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
