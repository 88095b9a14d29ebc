"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the TimeVQVAE hot path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import anything under `oracle/`, and only as the checker / CPU baseline.  The
product (`t-vq-vae-trajgen_amd/timevqvae`) never imports it and fails loudly when
its HIP library is missing.

Contents
  tvq_oracle.py  functional fp32 restatement (torch CPU) of the reference path,
                 each function citing the reference file:line it follows;
                 pinned by tests/golden/*.npz generated from the reference itself.
  vq_ref.c       plain-C restatement of the VQ assign (L2 + argmin) and EMA
                 update (vq.py:197-251), with an fp64 top-2 gap for near-tie
                 qualification; built into oracle/build/libvq_ref.so.
  rocket_ref.c   plain-C fp64 restatement of the ROCKET transform
                 (evaluation/rocket_functions.py:60-126), pthreads over examples for
                 the CPU baseline; built into oracle/build/librocket_ref.so.
"""
