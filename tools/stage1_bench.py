"""Time the Stage1 train step (config B: B=256,C=6,T=256,K=512) on the HIP path."""
import argparse, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch
from timevqvae.trainers import Stage1

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--B", type=int, default=256)
args = ap.parse_args()
dev = torch.device("cuda:0")
cfg = {
    "VQ-VAE": {"n_fft": 4, "codebook_sizes": {"lf": 512, "hf": 512}},
    "encoder": {"init_dim": 4, "hid_dim": 128, "n_resnet_blocks": 2, "downsampled_width": {"lf": 8, "hf": 32}},
    "decoder": {"n_resnet_blocks": 2},
    "exp_params": {"lr": 1e-3, "linear_warmup_rate": 0.1},
    "trainer_params": {"max_steps": {"stage1": 50000, "stage2": 200000}},
}
torch.manual_seed(0)
m = Stage1(256, 6, cfg).to(dev).train()
opt = m.configure_optimizers()["optimizer"]
g = torch.Generator().manual_seed(1234)
x = torch.cumsum(0.1 * torch.randn(args.B, 6, 256, generator=g), -1)
x = 2 * (x - x.amin(0, keepdim=True)) / (x.amax(0, keepdim=True) - x.amin(0, keepdim=True) + 1e-8) - 1
x = x.to(dev)

def step():
    opt.zero_grad()
    out = m.training_step((x, None), 0)
    out["loss"].sum().backward()
    opt.step()
    return out

for _ in range(args.warmup):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(args.steps):
    out = step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / args.steps
print(f"stage1 step: {dt*1e3:.2f} ms  ({1/dt:.1f} steps/s)  loss {float(out['loss'].sum()):.4f}")
