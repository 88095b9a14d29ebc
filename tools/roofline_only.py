"""Run only one roofline leg of bench.py (for rocprofv3 --pmc passes on that kernel).
usage: python tools/roofline_only.py [dominant|t32|wgrad|rbbwd|rb32bwd|linfwd|vqassign|attn|n16|rb64]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    leg = sys.argv[1] if len(sys.argv) > 1 else "dominant"
    fn = {"dominant": bench.dominant_leg, "t32": bench.conv_t32_leg,
          "wgrad": bench.conv_wgrad_leg, "rbbwd": bench.resblock_bwd_leg, "rb32bwd": bench.resblock_bwd32_leg,
          "linfwd": bench.linear_fwd_leg, "vqassign": bench.vq_assign_leg,
          "attn": bench.attn_branch_leg, "n16": bench.conv_n16_leg, "rb64": bench.rb64_fwd_leg}[leg]
    print(json.dumps(fn(torch.device("cuda", 0))))
