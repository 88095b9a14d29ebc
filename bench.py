"""bench.py — stage1+stage2 train steps/s on synthetic (B,C,T) trajectories (BASELINE.json).

One step = one stage1 VQ-VAE optimizer step + one stage2 MaskGIT optimizer step on a
B=256, C=6, T=256 synthetic batch with K=512 codebooks (BASELINE configs[1..3];
configs/config.yaml architecture otherwise).  N>1: one process per GPU, plain data
parallel (RCCL all-reduce of the flat gradient buffer, the reference's sync_codebook
EMA all-reduce), weak scaling (global batch 256*N).  Rank 0 prints ONE JSON line.
"""
import argparse
import copy
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
sys.path.insert(0, ROOT)

# kernel arguments in device memory (a HIP runtime option, read at its initialisation): the
# graph-replayed step's ~480 launches and the sampler's ~90 (same box, alternated processes:
# stage1 alone 2.80 -> 2.76-2.79 ms, sampler 4.71-4.73 -> 4.69-4.71 ms, joint within noise;
# profiles/r06_issue_order_ab.txt).  Inherited by the ranks bench.py launches.
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

B, C, T, K = 256, 6, 256, 512
N_CLASSES = 5


def config(sync):
    return {
        "VQ-VAE": {"n_fft": 4, "codebook_sizes": {"lf": K, "hf": K}, "sync_codebook": sync},
        "encoder": {"init_dim": 4, "hid_dim": 128, "n_resnet_blocks": 2,
                    "downsampled_width": {"lf": 8, "hf": 32}},
        "decoder": {"n_resnet_blocks": 2},
        "exp_params": {"lr": 1e-3, "linear_warmup_rate": 0.1},
        "trainer_params": {"max_steps": {"stage1": 50000, "stage2": 200000}},
        "MaskGIT": {
            "choice_temperatures": {"lf": 10, "hf": 4}, "T": {"lf": 10, "hf": 1},
            "prior_model_l": {"hidden_dim": 128, "n_layers": 4, "heads": 2, "ff_mult": 1,
                              "use_rmsnorm": True, "p_unconditional": 0.2, "model_dropout": 0.3,
                              "emb_dropout": 0.3},
            "prior_model_h": {"hidden_dim": 32, "n_layers": 1, "heads": 1, "ff_mult": 1,
                              "use_rmsnorm": True, "p_unconditional": 0.2, "model_dropout": 0.3,
                              "emb_dropout": 0.3},
            "cfg_scale": 1.0,
        },
        "fidelity_enhancer": {"dim": 8, "dim_mults": [1, 2, 4, 8], "resnet_block_groups": 4,
                              "dropout": 0.5, "tau_search_rng": [0.1, 0.5, 1, 2, 4],
                              "tau_search_subset_size": 1.0, "percept_loss_weight": 0.0},
    }


def synthetic_batch(seed, device):
    """random walk, min-max scaled per (c,t) to [-1,1]; y ~ U{0..4}."""
    g = torch.Generator().manual_seed(seed)
    x = torch.cumsum(0.1 * torch.randn(B, C, T, generator=g), -1)
    lo, hi = x.amin(0, keepdim=True), x.amax(0, keepdim=True)
    x = 2 * (x - lo) / (hi - lo + 1e-8) - 1
    y = torch.randint(0, N_CLASSES, (B, 1), generator=g)
    return x.to(device), y.to(device)


class JointTrainer:
    """stage1 step and stage2 step (stage2 trains on a frozen snapshot of stage1).

    The two steps are independent (the stage2 prior reads the frozen stage1, never the
    one being trained), so they run concurrently: stage1's LF and HF bands each do
    forward+backward on a side stream while stage2 runs on the current stream with its
    HF encoder / HF transformer on side streams (timevqvae.hip.streams).
    Graph mode (default), one replica: the step is one hipGraph
      [advance seed, zero_grad x2, stage1 LF | stage1 HF | stage2 fwd+bwd, AdamW1, AdamW2].
    Replicas (world > 1): stage1 and stage2 are captured as two graphs replayed on two
    streams (hip.graph.BranchStepGraph); each is followed on its stream by its own DP
    exchange (flat gradients + gates, BatchNorm statistics, stage1's sync_codebook
    statistics), so one stage's all-reduces run while the other's backward still computes;
    a final graph applies the codebook EMAs and both AdamW steps.  TVQ_DP_OVERLAP=0 keeps
    the previous form (one fwd+bwd graph, every exchange after it).  The LR schedulers run
    on the host before each replay.
    """

    def __init__(self, device, world, cfg=None, length=T, channels=C):
        from timevqvae.trainers import Stage1, Stage2
        from timevqvae.hip import rng
        from timevqvae.utils import set_seed
        set_seed(0)  # python / numpy (Snake a init) / torch
        rng.manual_seed(1)
        cfg = cfg if cfg is not None else config(world > 1)
        self.world = world
        self.s1 = Stage1(length, channels, cfg).to(device).train()
        s1_frozen = copy.deepcopy(self.s1)
        self.s2 = Stage2(None, None, length, channels, N_CLASSES, config=cfg,
                         stage1=s1_frozen).to(device).train()
        self.opt1 = self.s1.configure_optimizers()["optimizer"]
        self.opt2 = self.s2.configure_optimizers()["optimizer"]
        # the fixed zero_grad -> fwd+bwd -> step loop: each update zeroes the gradients it read,
        # so the next step's zero_grad launches nothing (hip/optim.py zero_after_step)
        self.opt1.zero_after_step = self.opt2.zero_after_step = True
        if world > 1:  # identical initial replicas (DDP semantics)
            for p in (self.opt1.flat, self.opt2.flat):
                dist.broadcast(p, 0)
            for m in (self.s1, self.s2):
                for b in m.buffers():
                    if b.is_floating_point():
                        dist.broadcast(b, 0)
        from timevqvae.hip.dp import ReplicaSync, flatten_bn_buffers
        self.sync = ReplicaSync(world)
        # BatchNorm running statistics of the trained modules, one flat buffer per stage
        # (stage1's encoders / decoders; the HF prior's Upscale): averaged over the replicas
        # every step, each right after its stage's backward
        self.bn_flat = ([flatten_bn_buffers([self.s1]),
                         flatten_bn_buffers([self.s2.maskgit.transformer_l,
                                             self.s2.maskgit.transformer_h])]
                        if world > 1 else [])
        self.device = device
        self._one = torch.ones((), device=device)
        self.graph = None
        self._pending = []
        self._scheds = (None, None)
        from timevqvae.hip.conv import PackCache
        on = os.environ.get("TVQ_PACK_CACHE", "1") != "0"
        self.packs = PackCache(device) if on else None
        # the DP form captures each stage as its own graph, each with its own cache
        self.packs12 = (PackCache(device), PackCache(device)) if on and world > 1 else (None, None)

    def _allreduce(self, opt):
        """DP exchange (timevqvae.hip.dp): mean of the flat gradients; the layer-dropout
        gates (which parameter segments some replica's forward used) are OR-ed (MAX), so
        every replica updates the same segments and the replicas stay identical."""
        self.sync.gradients(opt)

    def _sync_buffers(self, which=(0, 1)):
        """Mean of the BatchNorm running statistics over the replicas (DDP keeps them
        equal with broadcast_buffers; here every state_dict tensor stays bitwise equal).
        `which`: the stages whose buffers to average (the mean is elementwise, so averaging
        the stages separately gives the same bits as one buffer)."""
        for i in which:
            if i < len(self.bn_flat):
                self.sync.buffers(self.bn_flat[i])

    def _stage1_fwd_bwd(self, batch, packs):
        """Stage1 alone (the DP form's first branch): LF and HF bands forward+backward on
        their side streams, the codebook updates deferred.  Returns (out1, updates)."""
        import contextlib
        from timevqvae.hip import streams
        from timevqvae.hip.vq import deferred_codebook_updates
        with (packs.scope() if packs is not None else contextlib.nullcontext()), \
                streams.concurrent(), deferred_codebook_updates() as pend:
            hist1 = self.s1.forward_backward(batch, 0)
        return hist1(), pend

    def _stage2_fwd_bwd(self, batch, packs):
        """Stage2 alone (the DP form's second branch): forward+backward on the current
        stream with its HF chains on side streams."""
        import contextlib
        from timevqvae.hip import streams, wgrad
        from timevqvae.hip.conv import wgrad_deferred
        with (packs.scope() if packs is not None else contextlib.nullcontext()), \
                streams.concurrent():
            with wgrad_deferred(this_stream_only=True), wgrad.grouped():
                hist2 = self.s2.forward_backward(batch, self._one)
        return hist2()

    def _fwd_bwd(self, batch, defer, only=None, packs=None):
        """zero_grad, then stage1's LF and HF bands (forward+backward, one side stream
        each) || stage2 forward+backward on the current stream (with its own HF side
        streams); every stream is joined when the region ends.  only: "stage1" / "stage2"
        runs that stage alone (the bench's per-stage legs).
        Returns (out1, out2, deferred codebook updates)."""
        import contextlib
        from timevqvae.hip import streams, wgrad
        from timevqvae.hip.conv import wgrad_deferred
        from timevqvae.hip.vq import deferred_codebook_updates
        only = only or os.environ.get("TVQ_BENCH_ONLY")  # diagnosis: time one stage alone
        if only != "stage2":
            self.opt1.zero_grad()
        if only != "stage1":
            self.opt2.zero_grad()
        packs = packs if packs is not None else self.packs
        packs = packs.scope() if packs is not None else contextlib.nullcontext()
        with packs, streams.concurrent():
            with (deferred_codebook_updates() if defer else contextlib.nullcontext([])) as pend:
                # diagnosis only (TVQ_BENCH_BANDS=LF|HF): one stage1 band alone
                bands = tuple(os.environ.get("TVQ_BENCH_BANDS", "HF,LF").split(","))
                hist1 = self.s1.forward_backward(batch, 0, bands) if only != "stage2" else None
            if only != "stage1":
                # each prior backpropagated from its own loss on its own stream
                # (MaskGIT.forward_backward); Linear weight gradients: one grouped launch per
                # stream, the conv / norm weight-gradient reductions one batch per stream
                with wgrad_deferred(this_stream_only=True), wgrad.grouped():
                    hist2 = self.s2.forward_backward(batch, self._one)  # cached ones root
            else:
                hist2 = None
        return ((hist1() if hist1 else {"loss": torch.zeros(())}),
                (hist2() if hist2 else {"loss": torch.zeros(())}), pend)

    def step(self, batch):
        if self.graph is not None:
            outs = self.graph.replay()
            # StepGraph: the first segment returns (out1, out2); BranchStepGraph: one per stage
            return outs[0] if type(self.graph).__name__ == "StepGraph" else tuple(outs)
        from timevqvae.hip import rng
        rng.advance(self.device)
        out1, out2, _ = self._fwd_bwd(batch, defer=False)
        for opt in (self.opt1, self.opt2):
            opt.gather_gates()
            self._allreduce(opt)
            opt.step(gates_ready=True)
        self._sync_buffers()
        return out1, out2

    def stage_alone_ms(self, batch, which, steps=20, warmup=3):
        """One stage's optimizer step alone (the reference trains the stages one after the
        other), as its own hipGraph [advance seed, zero_grad, fwd+bwd (+ codebook EMA),
        AdamW] with its own weight-pack cache, replayed `steps` times after `warmup`: the
        per-stage reading beside the concurrent joint step.  World 1 only."""
        from timevqvae.hip import rng
        from timevqvae.hip.conv import PackCache
        from timevqvae.hip.graph import StepGraph
        opt = self.opt1 if which == "stage1" else self.opt2
        sch = self._scheds[0 if which == "stage1" else 1]
        packs = PackCache(self.device) if self.packs is not None else None

        def before():
            if sch is not None:
                sch.step()
            opt.push_lr()

        def seg():
            from timevqvae.hip import streams
            rng.advance(self.device)
            out = self._fwd_bwd(batch, False, only=which, packs=packs)
            opt.gather_gates()
            streams.join(backward_done=True)
            opt.step(lr_on_device=True, gates_ready=True)
            return out

        g = StepGraph([seg], [None], warmup=2, before=before).capture()
        for _ in range(warmup):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        del g
        torch.cuda.synchronize()
        return dt * 1e3

    def capture(self, batch):
        """Capture the step (runs 2 eager warmup steps first)."""
        from timevqvae.hip import rng
        from timevqvae.hip.graph import StepGraph
        scheds = (self.s1._sched, self.s2._sched)
        self._scheds = scheds
        self.s1._sched = self.s2._sched = None  # stepped on the host before each replay
        defer = self.world > 1  # sync_codebook all-reduce must sit between segments

        def before():
            for sch in scheds:
                if sch is not None:
                    sch.step()
            self.opt1.push_lr(self.opt2)  # both learning rates, one launch

        def seg1():
            rng.advance(self.device)
            out1, out2, self._pending = self._fwd_bwd(batch, defer)  # streams joined
            self.opt1.gather_gates()
            self.opt2.gather_gates()
            return out1, out2

        def between1():
            self._allreduce(self.opt1)
            self._allreduce(self.opt2)
            self._sync_buffers()
            for u in self._pending:
                u.reduce()

        def seg2():
            from timevqvae.hip.optim import step_pair
            for u in self._pending:
                u.apply()
            # both AdamW updates: two launches (tvq_adamw2) instead of four
            step_pair(self.opt1, self.opt2, lr_on_device=True, gates_ready=True)

        if self.world == 1 and os.environ.get("TVQ_ONE_GRAPH", "1") != "0":
            # one replica: nothing runs between the segments (no collectives, no deferred
            # codebook update), so the step is one graph
            from timevqvae.hip import streams

            def seg12():
                out = seg1()
                streams.join(backward_done=True)
                seg2()
                return out
            self.graph = StepGraph([seg12], [None], warmup=2, before=before).capture()
        elif os.environ.get("TVQ_DP_OVERLAP", "1") != "0":
            # replicas: stage1 and stage2 forward+backward as two graphs on two streams, each
            # followed at once by its own exchange (its stage's flat gradients + gates, its
            # BatchNorm statistics, for stage1 the sync_codebook statistics), so one stage's
            # all-reduces overlap the other stage's backward; then [codebook EMA, AdamW x2]
            from timevqvae.hip.graph import BranchStepGraph

            def branch1():
                rng.restart_calls()  # the seed advance itself runs eagerly before replay
                self.opt1.zero_grad()
                out1, self._pending = self._stage1_fwd_bwd(batch, self.packs12[0])
                self.opt1.gather_gates()
                return out1

            def after1():
                self._allreduce(self.opt1)
                self._sync_buffers((0,))
                for u in self._pending:
                    u.reduce()

            def branch2():
                self.opt2.zero_grad()
                out2 = self._stage2_fwd_bwd(batch, self.packs12[1])
                self.opt2.gather_gates()
                return out2

            def after2():
                self._allreduce(self.opt2)
                self._sync_buffers((1,))

            # stage2's forward+backward (~2.6 ms alone) ends before stage1's (~3.5 ms): its
            # exchange is issued first, so it runs while stage1 still computes
            self.graph = BranchStepGraph(lambda: rng.advance(self.device), [branch1, branch2],
                                         [after1, after2], seg2, warmup=2, before=before,
                                         replay_order=(1, 0)).capture()
        else:  # TVQ_DP_OVERLAP=0: one fwd+bwd graph, every exchange after it
            self.graph = StepGraph([seg1, seg2], [between1, None], warmup=2,
                                   before=before).capture()


class Stage1Trainer:
    """Stage1 alone (BASELINE configs[0]: T=128, K=256, configs/config.yaml widths), one
    hipGraph per step like JointTrainer: [advance seed, zero_grad, LF | HF fwd+bwd] ->
    [AdamW]."""

    def __init__(self, device, B_, T_, K_):
        from timevqvae.trainers import Stage1
        from timevqvae.hip import rng
        from timevqvae.hip.conv import PackCache
        from timevqvae.utils import set_seed
        set_seed(0)
        rng.manual_seed(1)
        cfg = config(False)
        cfg["VQ-VAE"]["codebook_sizes"] = {"lf": K_, "hf": K_}
        self.s1 = Stage1(T_, C, cfg).to(device).train()
        self.opt = self.s1.configure_optimizers()["optimizer"]
        self.device = device
        self.packs = PackCache(device)
        g = torch.Generator().manual_seed(1234)
        x = torch.cumsum(0.1 * torch.randn(B_, C, T_, generator=g), -1)
        x = 2 * (x - x.amin(0, keepdim=True)) / (x.amax(0, keepdim=True) - x.amin(0, keepdim=True) + 1e-8) - 1
        self.batch = (x.to(device), torch.randint(0, N_CLASSES, (B_, 1), generator=g).to(device))
        self.graph = None

    def capture(self):
        from timevqvae.hip import rng, streams
        from timevqvae.hip.graph import StepGraph
        sched = self.s1._sched
        self.s1._sched = None

        def before():
            sched.step()
            self.opt.push_lr()

        def seg1():
            rng.advance(self.device)
            self.opt.zero_grad()
            with self.packs.scope(), streams.concurrent():
                hist = self.s1.forward_backward(self.batch, 0)
            return hist()

        def seg2():
            self.opt.step(lr_on_device=True)

        self.graph = StepGraph([seg1, seg2], [None, None], warmup=2, before=before).capture()

    def timed(self, steps=20, warmup=3):
        for _ in range(warmup):
            self.graph.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            self.graph.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps


def config0_leg(device, cpu=True):
    """BASELINE configs[0] (stage1 VQ-VAE, T=128, K=256, config.yaml widths; the
    reference's CPU-runnable case) on the GPU at the config.yaml batch (32) and at 256,
    with the CPU port timed beside it (oracle/cpu_baseline.measure_stage1)."""
    out = {}
    for b in (32, 256):
        tr = Stage1Trainer(device, b, 128, 256)
        tr.capture()
        out[f"B{b}_ms_per_step"] = round(tr.timed() * 1e3, 3)
        del tr
    if cpu:
        from oracle import cpu_baseline
        threads = cpu_threads()
        for b in (32, 256):
            s = cpu_baseline.measure_stage1(threads, b, 128, 256, steps=5, warmup=2)
            out[f"cpu_B{b}_ms_per_step"] = round(s * 1e3, 1)
        out["cpu_cores"] = threads
    return out


# Algorithmic FLOPs of one joint step at B=256 (matmul/conv work of stage1 fwd+bwd and
# stage2 with every prior branch run): tools/count_step_flops.py over the CPU restatement
# of the same module tree -> profiles/r02_step_flops.json (169.78 GFLOP).
STEP_GFLOP = 169.78
# One sampler batch (BASELINE configs[4]: 1024 trajectories, 10 LF + 1 HF prior forwards and
# both decoders), counted the same way -> profiles/r03_step_flops.json.
SAMPLER_GFLOP_1024 = 375.0
# What the sampler batch executes (tools/count_step_flops.py `sampler_executed_gflop_per_1024`):
# the reference algorithm's count less the Linears the eval heads compose away while sampling
# (LF project_in folded into the embedding tables and project_out composed with pred_head's
# Linear; the HF project_in folded into Upscale's last
# conv and the token table, project_out composed with pred_head's Linear).
SAMPLER_EXEC_GFLOP_1024 = 334.8
# What the train step executes (tools/count_step_flops.py `step_executed_gflop_at_B256`): the
# algorithmic count less the Linears the priors' training forwards compose away (Upscale's last
# conv with the HF project_in's tl half, project_out with pred_head's Linear in both priors).
STEP_EXEC_GFLOP = 152.22
FP32_PEAK_TFLOPS = 157.3
HBM_PEAK_GBS = 8000.0


# PMC evidence of the roofline legs: profiles/<PROFILE_TAG>_<leg>_traffic.json, written by
# tools/gpu_roofline.sh + tools/roof_traffic.py on the tree named in its "tree" field
PROFILE_TAG = "r06"


def _traffic(leg):
    """(traffic bytes per op, evidence file, profiled tree) or (None, None, None)."""
    path = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_{leg}_traffic.json")
    if not os.path.exists(path):
        return None, None, None
    d = json.load(open(path))
    return d["traffic_bytes"], os.path.relpath(path, ROOT), d.get("tree")


def _with_traffic(res, leg):
    t, src, tree = _traffic(leg)
    res["traffic"] = t
    res["traffic_source"] = src
    res["traffic_tree"] = tree
    if t:
        res["traffic_over_algorithmic"] = round(t / res["algorithmic_bytes"], 3)
    return res


def cu_weighted_leg():
    """Sum of the step's algorithmic FLOPs over the summed device time of all its kernels
    (profiles/<PROFILE_TAG>_step_kernel_stats.csv, rocprofv3 over graph-replayed steps): the
    fraction of the fp32 peak the CUs deliver while busy, across all four streams."""
    path = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_step_kernel_stats.csv")
    if not os.path.exists(path):
        return None
    import csv
    rows = list(csv.DictReader(open(path)))
    us = sum(float(r["us_per_step"]) for r in rows)
    launches = sum(float(r["calls_per_step"]) for r in rows)
    tf = STEP_GFLOP / (us * 1e-3)  # GFLOP / ms = TFLOP/s
    return {"bound": "mfma", "gflop": STEP_GFLOP, "kernel_us_per_step": round(us, 1),
            "launches_per_step": launches, "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(tf / FP32_PEAK_TFLOPS, 4),
            "source": os.path.relpath(path, ROOT)}


def _graph_time_us(fns, reps):
    """Average device time per launch of `fns` (each called `reps` times, interleaved),
    captured in one hipGraph on a side stream and timed with HIP events recorded on that
    same stream (the host launch cost of the ctypes calls is not in the region)."""
    st = torch.cuda.Stream(device=torch.cuda.current_device())
    with torch.cuda.stream(st):
        for f in fns:
            f()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        gc.collect()
        gc.disable()  # see timevqvae.hip.graph.StepGraph.capture
        try:
            with torch.cuda.graph(g, stream=st):
                for _ in range(reps):
                    for f in fns:
                        f()
        finally:
            gc.enable()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(5):
            g.replay()
        e1.record(st)
        torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (5 * reps * len(fns))
    del g
    torch.cuda.synchronize()
    return us


def dominant_leg(device):
    """The step's top kernel by summed time (profiles/r03c_step_kernel_stats.csv:
    wgrad_wide_kernel, 4 launches and 239 us per step) and its largest single launch: the
    grouped weight gradient dW_i += dY_i^T X_i of every Linear of a prior, issued once
    at the end of its backward (timevqvae.hip.wgrad; 32x32x2 fp32 MFMA, 64x64 tiles, K =
    tokens split over 4 waves x S blocks) with its ordered slab sum wgrad_group_reduce_kernel
    (one op = these 2 launches).  Timed on the LF prior's set, accumulating into one flat
    gradient buffer as the step does: 4 layers x [q|k|v 384x128, out, ff1, ff2 128x128]
    over 6400 tokens (B=256 x 25) = 5.03 GFLOP and 4 * sum(K (M + N) + 2 M N) = 134.6 MB
    algorithmic per op (AI 37 FLOP/B: fp32 MFMA bound).  20 graph-replayed ops timed with
    HIP events on their stream."""
    from timevqvae.hip import wgrad
    K = 6400
    shapes = [(384, 128), (128, 128), (128, 128), (128, 128)] * 4
    flat = torch.zeros(sum(m * n for m, n in shapes), device=device)
    recs, off = [], 0
    for M, N in shapes:
        dy = torch.randn(K, M, device=device)
        x = torch.randn(K, N, device=device)
        recs.append((dy, M, x, N, flat[off:off + M * N], N, M, N, K))
        off += M * N
    fn = (lambda: wgrad.launch(recs))
    with torch.no_grad():
        us = _graph_time_us([fn], 20)
    flops = sum(2.0 * K * M * N for M, N in shapes)
    byts = sum(4.0 * (K * (M + N) + 2 * M * N) for M, N in shapes)
    tf = flops / (us * 1e-6) / 1e12
    return _with_traffic({"bound": "mfma", "kernel": "wgrad_wide_kernel + wgrad_group_reduce_kernel (grouped "
                                       "weight gradients of the LF prior's 16 Linears, "
                                       "dW_i += dY_i^T X_i over 6400 tokens, fp32 MFMA)",
            "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / FP32_PEAK_TFLOPS, 4),
            "algorithmic_bytes": byts, "flops_per_launch": flops, "avg_launch_us": round(us, 2),
            "hbm_frac": round(byts / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}, "dominant")


def conv_wgrad_leg(device):
    """The LF band's 64 -> 64 3x3 conv weight (+ bias) gradient on (256, 64, 3, 8) (12
    launches per step): dW[64][577] = sum over 6144 positions of dY x im2col(X) ->
    2 * 6144 * 64 * 577 = 453.8 MFLOP and 4 * (2 * 6144 * 64 + 64 * 577) = 3.29 MB
    algorithmic per op (AI 138 FLOP/B: fp32 MFMA bound).  One op = conv_wgrad_w8_kernel
    (16 images per block, the 4 waves' partial tiles summed in LDS; 16 slab rows) + its
    ordered slab sum (batched at the band's end in the step; here after each op).  50
    graph-replayed ops timed with HIP events."""
    from timevqvae.hip._native import call, ptr, stream_ptr, value
    B, C, H, W, Co = 256, 64, 3, 8, 64
    x = torch.randn(B, C, H, W, device=device)
    dy = torch.randn(B, Co, H, W, device=device)
    dw = torch.zeros(Co, C, 3, 3, device=device)
    db = torch.zeros(Co, device=device)
    ws = torch.empty(value("tvq_conv_workspace", 4, B, C, H, W, Co, 3, 3, 1, 0), device=device)
    fn = (lambda: call("tvq_conv2d_wgrad", ptr(x), B, C, H, W, ptr(dy), Co, W, 3, 3, 1, 0, ptr(dw),
                       ptr(db), 1, ptr(ws), stream_ptr()))
    with torch.no_grad():
        us = _graph_time_us([fn], 50)
    flops = 2.0 * B * H * W * Co * (C * 9 + 1)
    byts = 4.0 * (2 * B * H * W * C + Co * (C * 9 + 1))
    tf = flops / (us * 1e-6) / 1e12
    return _with_traffic({"bound": "mfma", "kernel": "conv_wgrad_w8_kernel<8,8> + its ordered slab sum (LF "
                                       "64->64 3x3 conv weight+bias gradient over 6144 positions, "
                                       "16 images per block, fp32 MFMA)",
            "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / FP32_PEAK_TFLOPS, 4),
            "algorithmic_bytes": byts, "flops_per_launch": flops, "avg_launch_us": round(us, 2),
            "hbm_frac": round(byts / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}, "wgrad")


def resblock_bwd32_leg(device):
    """The same op at C = 32 on (256, 32, 3, 16) (the LF band's level-3 ResBlocks, 4 ops per
    step), where round 6 replaced the per-image C x (9C+1) slab rows (37 KB per image per
    conv, 12x the image's activations) by the g / s operand planes and one image-batched
    weight-gradient launch (conv_wgrad_w16: both convs' dW|db over 16-image blocks): rb_bwd2
    + rb_bwd1 + conv_wgrad_w16 + the batched ordered sum of its 16-row slabs.  Algorithmic
    work as resblock_bwd_leg's formula: 4 * 2 * 256*48*32*288 (+bias) = 0.906 GFLOP;
    bytes 4 * B*C*P*4 + weights = 6.37 MB."""
    return resblock_bwd_leg(device, C=32, W=16, leg="rb32bwd")


def resblock_bwd_leg(device, C=16, W=32, leg="rbbwd"):
    """The round-3a top kernel by summed time (profiles/r03a_step_kernel_stats.csv): the fused
    ResBlock backward (csrc/tvq_resblock.hip rb_bwd2 + rb_bwd1, reference vq_vae.py:13-62) at
    its most frequent shape, C = 16 on (256, 16, 3, 32) (8 ops per step).  One op = rb_bwd2
    (dropout' -> conv2 weight gradient slab row + data gradient -> Snake' -> per-image BN
    backward partials and Snake a2 term) + rb_bwd1 (every block reduces those partials to
    the BN coefficients -> BN' -> conv1 weight gradient + data gradient -> Snake' + identity
    skip, per-image Snake a1 term) + one batched launch of the four ordered slab sums
    (dW2|db2, dW1|db1, da1, da2: as in the step, where they join the band-end batch).
    Algorithmic work per op: two 3x3 data gradients 2 * B*P*C*9C each and two weight+bias
    gradients 2 * B*P*C*(9C+1) each (P = 3W positions) = 4 * 2 * 256*96*16*144 (+bias) =
    453.8 MFLOP; bytes: dy, x, h read and dx written (4 * B*C*P*4 B) + both weights read and
    their gradients written = 6.33 MB (AI 72 FLOP/B: fp32 MFMA bound).  50 graph-replayed ops
    timed with HIP events on their stream."""
    from timevqvae.hip import rng
    from timevqvae.hip._native import call, ptr, stream_ptr, value
    B, H = 256, 3
    P = H * W
    g = torch.Generator(device="cpu").manual_seed(5)
    rnd = lambda *sh, s=1.0: (torch.randn(*sh, generator=g) * s).to(device)  # noqa: E731
    x, dy = rnd(B, C, H, W), rnd(B, C, H, W)
    a1 = (0.2 + 0.3 * torch.rand(C, generator=g)).to(device)
    a2 = (0.2 + 0.3 * torch.rand(C, generator=g)).to(device)
    w1, w2 = rnd(C, C, 3, 3, s=0.1), rnd(C, C, 3, 3, s=0.1)
    b1, b2 = rnd(C, s=0.1), rnd(C, s=0.1)
    bw, bb = torch.ones(C, device=device), torch.zeros(C, device=device)
    rm, rv = torch.zeros(C, device=device), torch.ones(C, device=device)
    nbt = torch.zeros((), dtype=torch.int64, device=device)
    h, y = torch.empty_like(x), torch.empty_like(x)
    save = torch.empty(4 * C, device=device)
    ws = torch.empty(value("tvq_resblock_workspace", B, C, H, W), device=device, dtype=torch.uint8)
    seed = rng.seed_tensor(device)
    call("tvq_resblock_train_fwd", ptr(x), B, C, H, W, ptr(a1), ptr(w1), ptr(b1), ptr(bw),
         ptr(bb), ptr(rm), ptr(rv), ptr(nbt), 0.1, 1e-5, ptr(a2), ptr(w2), ptr(b2), 0.3,
         ptr(seed), 0, ptr(h), ptr(y), ptr(save), ptr(ws), stream_ptr())
    dx = torch.empty_like(x)
    grads = [torch.zeros(t.shape, device=device) for t in (a1, w1, b1, bw, bb, a2, w2, b2)]

    def fn():  # as in the step: the slab sums deferred to one batched launch at the end
        call("tvq_conv_wgrad_defer_begin")
        call("tvq_resblock_bwd", ptr(dy), ptr(x), ptr(h), B, C, H, W, ptr(a1), ptr(w1), ptr(bw),
             ptr(save), ptr(a2), ptr(w2), 0.3, ptr(seed), 0, ptr(dx), *[ptr(t) for t in grads],
             1, ptr(ws), stream_ptr())
        call("tvq_conv_wgrad_defer_flush", stream_ptr())
    with torch.no_grad():
        us = _graph_time_us([fn], 50)
    K = 9 * C
    flops = 2.0 * (2.0 * B * P * C * K) + 2.0 * (2.0 * B * P * C * (K + 1))
    byts = 4.0 * (4 * B * C * P + 2 * (C * K + C) + 2 * (C * K + C))
    tf = flops / (us * 1e-6) / 1e12
    kern = (f"fused ResBlock backward, C={C} on (256,{C},3,{W}): rb_bwd2_kernel + "
            f"rb_bwd1_kernel<RB<{C},{W}>> + one batched ordered slab-sum launch (16x16x4 fp32 "
            f"MFMA, 8 waves per image)") if leg == "rbbwd" else (
            f"fused ResBlock backward, C={C} on (256,{C},3,{W}): rb_bwd2_kernel + rb_bwd1_kernel"
            f"<RB<{C},{W}>> writing the g / s planes + conv_wgrad_w8_kernel<16,8> (both weight "
            f"gradients, 16 images per block) + the batched ordered sum of its 16-row slabs")
    return _with_traffic({"bound": "mfma", "kernel": kern,
            "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / FP32_PEAK_TFLOPS, 4),
            "algorithmic_bytes": byts, "flops_per_launch": flops, "avg_launch_us": round(us, 2),
            "launches_per_op": 3 if leg == "rbbwd" else 4,
            "hbm_frac": round(byts / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}, leg)


def vq_assign_leg(device):
    """The VQ codebook assignment vq_assign_kernel (the step's top kernel by summed time in
    profiles/r03b_step_kernel_stats.csv, second in r03c: 4 launches, 192 us per step) (csrc/tvq_vq.hip; reference vq.py:205-222
    EuclideanCodebook: dist = -(|x|^2 - 2 x E^T + |E|^2), argmax), at the HF band's training
    shape: the (256, 128, 3, 32) NCHW latent read as (B, 96 tokens, D = 128) through its
    strides against K = 512 codes, straight-through output, commit partials and the token-
    major copy for the EMA statistics (tvq_vq_assign_rows, as hip.vq.vq runs it).
    Algorithmic work per launch: 2 M K D = 2 x 24576 x 512 x 128 = 3.22 GFLOP; bytes: x read,
    E read, quantised x written, int64 + int32 indices = 4 (2 M D + K D) + 12 M = 25.7 MB
    (AI 125 FLOP/B: fp32 MFMA bound).  50 graph-replayed launches timed with HIP events."""
    from timevqvae.hip._native import call, ptr, stream_ptr, value
    B, D, H, W, K = 256, 128, 3, 32, 512
    N = H * W
    M = B * N
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(B, D, H, W, generator=g).to(device)
    E = torch.randn(K, D, generator=g).to(device)
    ee = torch.empty(K, device=device)
    call("tvq_vq_sqnorm", ptr(E), K, D, ptr(ee), stream_ptr())
    out = torch.empty_like(x)
    idx = torch.empty(M, device=device, dtype=torch.long)
    idx32 = torch.empty(M, device=device, dtype=torch.int32)
    part = torch.empty(value("tvq_vq_assign_nblocks", M), device=device)
    rows = torch.empty(M, D, device=device)
    sB, sN, sD = D * N, 1, N  # the token view (B, N, D) of the NCHW latent
    fn = (lambda: call("tvq_vq_assign_rows", ptr(x), B, N, D, sB, sN, sD, ptr(E), ptr(ee), K, 1,
                       0.0, None, None, 0, ptr(out), ptr(idx), ptr(idx32), ptr(part), ptr(rows),
                       stream_ptr()))
    with torch.no_grad():
        us = _graph_time_us([fn], 50)
    flops = 2.0 * M * K * D
    byts = 4.0 * (2 * M * D + K * D) + 12.0 * M
    tf = flops / (us * 1e-6) / 1e12
    return _with_traffic({"bound": "mfma", "kernel": "vq_assign_kernel<128,false>: HF codebook assignment, "
                                       "24576 token rows x 512 codes x D 128, 16x16x4 fp32 "
                                       "MFMA distances + running argmax, straight-through "
                                       "output, token-major copy for the EMA statistics",
            "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / FP32_PEAK_TFLOPS, 4),
            "algorithmic_bytes": byts, "flops_per_launch": flops, "avg_launch_us": round(us, 2),
            "hbm_frac": round(byts / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}, "vqassign")


def linear_fwd_leg(device):
    """The LF prior's Linear forward at its training shape (gemm_rb2_kernel<64, true>: 14 of
    its 15 launches per step are this shape): Y = R + X W^T + b over the 6400 token rows of
    the stage2 batch (B = 256 x 25 tokens), K = N = 128 (hidden 128, ff_mult 1; reference
    bidirectional_transformer.py / x-transformers Linear).  Algorithmic work per launch:
    2 M N K = 209.7 MFLOP; bytes X, W, b, R read and Y written = 4 (M K + N K + N + 2 M N) =
    9.9 MB (AI 21 FLOP/B: at the fp32 MFMA / HBM ridge).  50 graph-replayed launches timed
    with HIP events on their stream."""
    from timevqvae.hip.linear import gemm
    M, N, K = 6400, 128, 128
    g = torch.Generator(device="cpu").manual_seed(6)
    x = torch.randn(M, K, generator=g).to(device)
    w = (torch.randn(N, K, generator=g) * 0.05).to(device)
    b = (torch.randn(N, generator=g) * 0.1).to(device)
    r = torch.randn(M, N, generator=g).to(device)
    y = torch.empty(M, N, device=device)
    fn = (lambda: gemm(x, K, 1, w, 1, K, M, N, K, out=y, ldc=N, bias=b, R=r, ldr=N))
    with torch.no_grad():
        us = _graph_time_us([fn], 50)
    flops = 2.0 * M * N * K
    byts = 4.0 * (M * K + N * K + N + 2 * M * N)
    tf = flops / (us * 1e-6) / 1e12
    return _with_traffic({"bound": "mfma", "kernel": "gemm_rb2_kernel<64,true>: LF prior Linear forward "
                                       "Y = R + X W^T + b, (6400 x 128) x (128 x 128), "
                                       "32x32x2 fp32 MFMA, one 32x32 tile per wave",
            "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / FP32_PEAK_TFLOPS, 4),
            "algorithmic_bytes": byts, "flops_per_launch": flops, "avg_launch_us": round(us, 2),
            "hbm_frac": round(byts / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}, "linfwd")


def attn_branch_leg(device):
    """The LF prior's fused attention branch forward (csrc/tvq_xattn.hip, round 5; reference
    bidirectional_transformer.py:92-110): RMSNorm + QKV + 2-head softmax attention (dropout
    0.3) + gated out-projection + residual for 256 sequences of 25 tokens, one launch.
    Algorithmic work: QKV 2*6400*128*384 + scores and P V 2 heads * 256 * 2 * (2*25*25*64) +
    out-projection 2*6400*128*128 = 920.6 MFLOP; bytes: x read, the 4 weights read, y, xn,
    qkv, o written (+ inv, lse) = 23.4 MB (AI 39 FLOP/B: fp32 MFMA bound).  50 graph-replayed
    launches timed with HIP events on their stream."""
    import math
    from timevqvae.hip import rng
    from timevqvae.hip._native import call, ptr, stream_ptr
    B, S, D = 256, 25, 128
    M = B * S
    g = torch.Generator(device="cpu").manual_seed(11)
    rnd = lambda *sh, s=1.0: (torch.randn(*sh, generator=g) * s).to(device)  # noqa: E731
    x, W, Wo, gn = rnd(M, D), rnd(3 * D, D, s=0.08), rnd(D, D, s=0.08), 1 + rnd(D, s=0.1)
    gate = torch.ones(1, device=device)
    seed = rng.seed_tensor(device)
    y, xn, o = (torch.empty(M, D, device=device) for _ in range(3))
    inv = torch.empty(M, device=device)
    qkv = torch.empty(M, 3 * D, device=device)
    lse = torch.empty(B * 2 * S, device=device)
    fn = (lambda: call("tvq_attn_branch_fwd", ptr(x), B, S, D, 2, ptr(gn), math.sqrt(D), ptr(W),
                       ptr(Wo), ptr(gate), 0.3, ptr(seed), 0, ptr(y), ptr(xn), ptr(inv), ptr(qkv),
                       ptr(o), ptr(lse), stream_ptr()))
    with torch.no_grad():
        us = _graph_time_us([fn], 50)
    flops = 2.0 * M * D * 3 * D + 2 * B * 2 * (2 * S * S * 64) + 2.0 * M * D * D
    byts = 4.0 * (M * D + 4 * D * D + D + 3 * M * D + 3 * M * D + M + B * 2 * S)
    tf = flops / (us * 1e-6) / 1e12
    return _with_traffic({"bound": "mfma", "kernel": "xattn_fwd_kernel: fused LF prior attention "
                                       "branch (RMSNorm + QKV + attention + gated out-projection"
                                       " + residual), 256 x 25 tokens, 32x32x2 fp32 MFMA",
            "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / FP32_PEAK_TFLOPS, 4),
            "algorithmic_bytes": byts, "flops_per_launch": flops, "avg_launch_us": round(us, 2),
            "hbm_frac": round(byts / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}, "attn")


def conv_n16_leg(device):
    """The HF decoder ResBlock(128 -> 16)'s 3x3 conv on (256, 128, 3, 32) on the few-output
    wide-input kernel (conv_n16_kernel, round 5): 2 * 24576 * 16 * 1152 = 906.0 MFLOP;
    bytes: input 12.58 MB read + output 1.57 MB written + weight = 14.2 MB (AI 64 FLOP/B).
    50 graph-replayed launches inside a pack-cache scope (the weight packed once, as in the
    step) timed with HIP events."""
    from timevqvae.hip._native import call, ptr, stream_ptr, value
    B, C, H, W, N = 256, 128, 3, 32, 16
    g = torch.Generator(device="cpu").manual_seed(12)
    x = torch.randn(B, C, H, W, generator=g).to(device)
    w = (torch.randn(N, C, 3, 3, generator=g) * 0.03).to(device)
    b = torch.zeros(N, device=device)
    y = torch.empty(B, N, H, W, device=device)
    ws = torch.empty(value("tvq_conv_workspace", 0, B, C, H, W, N, 3, 3, 1, 0), device=device)
    fn = (lambda: call("tvq_conv2d_fwd", ptr(x), B, C, H, W, ptr(w), ptr(b), N, 3, 3, 1, 0, ptr(y),
                       None, 0.0, None, 0, ptr(ws), stream_ptr()))
    from timevqvae.hip.conv import PackCache
    cache = PackCache(device, floats=1 << 20)
    with torch.no_grad(), cache.scope():
        us = _graph_time_us([fn], 50)
    flops = 2.0 * B * H * W * N * C * 9
    byts = 4.0 * (B * C * H * W + B * N * H * W + N * C * 9)
    tf = flops / (us * 1e-6) / 1e12
    return _with_traffic({"bound": "mfma", "kernel": "conv_n16_kernel<F,3,3>: HF 128->16 3x3 conv "
                                       "on (256,128,3,32), one image per 8-wave block, 16x16x4 "
                                       "fp32 MFMA (weight packed once by the pack cache)",
            "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / FP32_PEAK_TFLOPS, 4),
            "algorithmic_bytes": byts, "flops_per_launch": flops, "avg_launch_us": round(us, 2),
            "hbm_frac": round(byts / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}, "n16")


def rb64_fwd_leg(device):
    """The LF band's fused ResBlock(64, 64) training forward on (256, 64, 3, 8)
    (csrc/tvq_resblock_w8.hip, round 5; vq_vae.py:13-62): w8_fwd1 + the BN finish +
    w8_fwd2 (3 launches; the weights packed once by a pack-cache scope).  Algorithmic work: two 3x3 convs 2 * 2*6144*64*576 = 906.0 MFLOP;
    bytes: x read, y written, h / Snake_a1(x) / Snake_a2(BN(h)) written for the backward and
    both weights read = 4 * (5 * 393216 + 2 * 36928) = 8.16 MB.  50 graph-replayed ops."""
    from timevqvae.hip import rng
    from timevqvae.hip._native import call, ptr, stream_ptr, value
    B, C, H, W = 256, 64, 3, 8
    g = torch.Generator(device="cpu").manual_seed(13)
    x = torch.randn(B, C, H, W, generator=g).to(device)
    a1 = (0.2 + 0.3 * torch.rand(C, generator=g)).to(device)
    a2 = (0.2 + 0.3 * torch.rand(C, generator=g)).to(device)
    w1 = (torch.randn(C, C, 3, 3, generator=g) * 0.04).to(device)
    w2 = (torch.randn(C, C, 3, 3, generator=g) * 0.04).to(device)
    b1, b2 = torch.zeros(C, device=device), torch.zeros(C, device=device)
    bw, bb = torch.ones(C, device=device), torch.zeros(C, device=device)
    rm, rv = torch.zeros(C, device=device), torch.ones(C, device=device)
    nbt = torch.zeros((), dtype=torch.int64, device=device)
    h = torch.empty(value("tvq_resblock_saved_floats", B, C, H, W), device=device)
    y = torch.empty_like(x)
    save = torch.empty(4 * C, device=device)
    ws = torch.empty(value("tvq_resblock_workspace", B, C, H, W), device=device, dtype=torch.uint8)
    seed = rng.seed_tensor(device)
    fn = (lambda: call("tvq_resblock_train_fwd", ptr(x), B, C, H, W, ptr(a1), ptr(w1), ptr(b1),
                       ptr(bw), ptr(bb), ptr(rm), ptr(rv), ptr(nbt), 0.1, 1e-5, ptr(a2), ptr(w2),
                       ptr(b2), 0.3, ptr(seed), 0, ptr(h), ptr(y), ptr(save), ptr(ws), stream_ptr()))
    from timevqvae.hip.conv import PackCache
    cache = PackCache(device, floats=1 << 20)
    with torch.no_grad(), cache.scope():  # the weights packed once, as in the step
        us = _graph_time_us([fn], 50)
    flops = 2.0 * (2.0 * B * H * W * C * 9 * C)
    byts = 4.0 * (5 * B * C * H * W + 2 * (C * C * 9 + C))
    tf = flops / (us * 1e-6) / 1e12
    return _with_traffic({"bound": "mfma", "kernel": "w8_fwd1_kernel + bn_stats_final_kernel + "
                                       "w8_fwd2_kernel: fused LF ResBlock(64,64) training forward "
                                       "on (256,64,3,8), one image per 8-wave block, weights from "
                                       "L2, 32x32x2 fp32 MFMA",
            "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / FP32_PEAK_TFLOPS, 4), "launches_per_op": 3,
            "algorithmic_bytes": byts, "flops_per_launch": flops, "avg_launch_us": round(us, 2),
            "hbm_frac": round(byts / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}, "rb64")


def roofline_leg(device, ms_per_step):
    """bench JSON `roofline`: the step's top kernel by summed time in the committed step
    table (profiles/r05_step_kernel_stats.csv: conv_t32_kernel<F,3,3>, the HF 128 -> 128
    3x3 conv, 2 launches and 158 us per step; conv_t32_leg) at top level (also under
    `conv_t32`); the grouped Linear weight gradients of the LF prior (`wgrad_group`,
    dominant_leg: the top kernel of rounds 3-4); the VQ codebook assignment (`vq_assign`);
    the fused ResBlock backward (`resblock_bwd`, resblock_bwd_leg); the LF prior's Linear
    forward (`linear_fwd`); the LF 64-channel conv weight gradient (`conv_wgrad`,
    conv_wgrad_leg); the whole step against the fp32 MFMA peak (`step`)."""
    t32 = conv_t32_leg(device)
    out = dict(t32)
    out["conv_t32"] = t32
    out["wgrad_group"] = dominant_leg(device)
    out["vq_assign"] = vq_assign_leg(device)
    out["resblock_bwd"] = resblock_bwd_leg(device)
    out["resblock_bwd32"] = resblock_bwd32_leg(device)
    out["linear_fwd"] = linear_fwd_leg(device)
    out["conv_wgrad"] = conv_wgrad_leg(device)
    tf = STEP_GFLOP / ms_per_step  # GFLOP / ms = TFLOP/s
    out["step"] = {"bound": "mfma", "gflop": STEP_GFLOP, "achieved": round(tf, 2),
                   "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                   "frac": round(tf / FP32_PEAK_TFLOPS, 4),
                   "executed_gflop": STEP_EXEC_GFLOP,
                   "executed_frac": round(STEP_EXEC_GFLOP / ms_per_step / FP32_PEAK_TFLOPS, 4),
                   "source": "tools/count_step_flops.py -> profiles/r05_step_flops.json (step_gflop_at_B256)"}
    out["step_frac"] = out["step"]["frac"]
    out["cu_weighted"] = cu_weighted_leg()
    out["attn_branch"] = attn_branch_leg(device)
    out["conv_n16"] = conv_n16_leg(device)
    out["rb64_fwd"] = rb64_fwd_leg(device)
    return out


def conv_t32_leg(device):
    """Average duration of the largest conv op at its step shape, on the stream it runs on
    (HIP events), with its algorithmic FLOPs -> achieved / peak.

    The op is the HF encoder ResBlock(16->128) second conv, (256,128,3,32) x (128,128,3,3):
    the largest single conv of the step (7.25 GFLOP).  As in the step it
    runs as one conv_t32_kernel launch (128-channel x 96-position tile on the 32x32x2 fp32
    MFMA, no split-K) reading the weight the step's pack cache packed once at the scope's
    begin (hip.conv.PackCache).  The committed rocprofv3 summary
    (profiles/<PROFILE_TAG>_t32_kernel_stats.csv) lists the launches; `traffic` is the
    PMC-measured HBM bytes per op from profiles/<PROFILE_TAG>_t32_traffic.json (FETCH_SIZE x2 +
    WRITE_SIZE passes on the tree its "tree" field names)."""
    from timevqvae.hip.conv import PackCache, conv2d
    x = torch.randn(256, 128, 3, 32, device=device)
    w = torch.randn(128, 128, 3, 3, device=device) * 0.03
    b = torch.zeros(128, device=device)
    cache = PackCache(device, floats=1 << 20)
    with cache.scope():
        for _ in range(3):
            conv2d(x, w, b)
    with cache.scope():  # the weight is packed here, once; the timed launches only convolve
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record(st)
        for _ in range(n):
            conv2d(x, w, b)
        e1.record(st)
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    flops = 2.0 * (256 * 3 * 32) * 128 * (128 * 9)
    achieved = flops / (ms * 1e-3) / 1e12
    return _with_traffic({"bound": "mfma", "kernel": "conv2d 128->128 3x3 @ (256,128,3,32): "
                                       "conv_t32_kernel<F,3,3,1,BK64,NW12> (32x32x2 fp32 MFMA; "
                                       "weight packed once per step by the pack cache)",
            "achieved": round(achieved, 2), "peak": 157.3, "unit": "TFLOP/s",
            "frac": round(achieved / 157.3, 4),
            "algorithmic_bytes": 4 * (256 * 128 * 3 * 32 * 2 + 128 * 128 * 9),
            "avg_launch_ms": round(ms, 4), "avg_launch_us": round(ms * 1e3, 2),
            "flops_per_launch": flops}, "t32")


def sampler_leg(tr, device, num=1024, reps=5, graph_reps=20, world=1):
    """BASELINE configs[4]: MaskGIT iterative decoding (LF 10 steps + HF 1 step) of `num`
    trajectories + LF/HF decoding to (num, 6, 256), with the bench's stage2 weights
    (tools/sampler_bench.py is the standalone version with a CPU baseline).  At world > 1
    every rank runs its own replica of the graphed batch at the same time (sampling does not
    shard: N GPUs are N replicas, configs[4]'s "8 GPU throughput"): barrier, `graph_reps`
    replays, barrier, the max elapsed over the ranks -> aggregate trajectories/s."""
    mg = tr.s2.maskgit
    was = mg.training
    mg.eval()

    def run():
        s_l, s_h = mg.iterative_decoding(num=num, device=device)
        return mg.decode_token_ind_to_timeseries(s_l, "lf") + \
            mg.decode_token_ind_to_timeseries(s_h, "hf")

    from timevqvae.models import FidelityEnhancer
    from timevqvae.utils.sample_utils import GraphedSampler
    fe = FidelityEnhancer(T, C, config(False)).to(device).eval()

    def timed(fn, n=reps, sync_ranks=False):
        fn()  # (a GraphedSampler captures here)
        fn()
        torch.cuda.synchronize()
        if sync_ranks:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(n):
            out = fn()
        torch.cuda.synchronize()
        if sync_ranks:
            dist.barrier()
        dt = (time.perf_counter() - t0) / n
        if sync_ranks:
            t = torch.tensor([dt], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t)
        return dt, out

    with torch.no_grad():
        dt_eager, x_new = timed(run)
        dt_fe, _ = timed(lambda: fe(x_new))
    # the whole batch as one hipGraph (GraphedSampler), without and with the FE
    dt, _ = timed(GraphedSampler(mg, num, device).sample, graph_reps, sync_ranks=world > 1)
    dt_g_fe, _ = timed(GraphedSampler(mg, num, device, fidelity_enhancer=fe).sample, graph_reps,
                       sync_ranks=world > 1)
    mg.train(was)
    # the reference's TrainedModelSampler.sample = decode + FidelityEnhancer (sampler.py:141-169)
    gflop = SAMPLER_GFLOP_1024 * num / 1024
    gexec = SAMPLER_EXEC_GFLOP_1024 * num / 1024
    roof = {"bound": "mfma", "gflop": round(gflop, 2), "achieved": round(gflop / (dt * 1e3), 2),
            "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(gflop / (dt * 1e3) / FP32_PEAK_TFLOPS, 4),
            "frac_counts": "the reference algorithm's FLOPs (what the batch computes, as the "
                           "reference would)",
            "executed_gflop": round(gexec, 2),
            "executed_frac": round(gexec / (dt * 1e3) / FP32_PEAK_TFLOPS, 4),
            "executed_counts": "the FLOPs the folded eval heads actually execute",
            "source": "tools/count_step_flops.py -> profiles/r05_step_flops.json "
                      "(sampler_gflop_per_1024, sampler_executed_gflop_per_1024)"}
    out = {"num": num, "ms_per_batch": round(dt * 1e3, 3), "roofline": roof,
           "trajectories_per_s": round(num / dt, 1), "reps": graph_reps, "eager_reps": reps,
           "launch": "hipgraph",
           "eager_ms_per_batch": round(dt_eager * 1e3, 3),
           "fidelity_enhancer_ms": round(dt_fe * 1e3, 3),
           "with_fe_ms_per_batch": round(dt_g_fe * 1e3, 3),
           "with_fe_trajectories_per_s": round(num / dt_g_fe, 1)}
    if world > 1:
        out.update({"replicas": world, "ms_per_batch_is": "max over the ranks, all replicas "
                                                           "sampling at once",
                    "aggregate_trajectories_per_s": round(world * num / dt, 1),
                    "aggregate_with_fe_trajectories_per_s": round(world * num / dt_g_fe, 1)})
    return out


def host_cpus():
    """(CPUs this process may run on = len(sched_getaffinity), the cgroup CPU quota in CPUs
    or None when unlimited)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return aff, quota


def cpu_threads():
    """Torch threads of the CPU legs: TVQ_CPU_THREADS, else the CPUs this process can use
    (the host's cores) = its affinity mask, capped by the cgroup CPU quota.  On
    the GPU box the mask holds all 256 CPUs of the EPYC 9575F pair but the quota is 16 CPUs,
    and the port's joint step measured 0.69 / 1.07 / 2.29 s at 16 / 32 / 64 threads there
    (profiles/r06_cpu_threads_probe.txt): threads beyond the quota only wait for it."""
    if "TVQ_CPU_THREADS" in os.environ:
        return int(os.environ["TVQ_CPU_THREADS"])
    aff, quota = host_cpus()
    return max(1, min(aff, int(quota))) if quota else aff


def cpu_baseline_leg():
    """the CPU port of the joint step (oracle/cpu_baseline.py, every
    reference dropout on) on the CPUs this process may use (cpu_threads): 2 untimed warmups,
    then the median of 5 timed steps; the CPU model, the affinity mask size and the cgroup
    quota are recorded.  The port is checked against the reference's own CPU step in the
    build container (tools/cpu_ref_compare.py -> profiles/r06_cpu_ref_compare.json)."""
    from oracle import cpu_baseline
    aff, quota = host_cpus()
    threads = cpu_threads()
    med, ts = cpu_baseline.measure(threads, steps=5, warmup=2, detail=True)
    return {"value": round(1.0 / med, 4), "unit": "steps/s", "cores": threads, "kind": "port",
            "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "cpu_model": cpu_baseline.cpu_model(),
            "step_s": [round(t, 4) for t in ts],
            "sample": f"median of 5 timed joint steps (after 2 untimed warmups) of "
                      f"oracle/cpu_baseline.py at B=256,C=6,T=256,K=512, every reference "
                      f"dropout on, on {threads} torch threads = the CPUs this process may use "
                      f"(affinity mask {aff} CPUs capped by the cgroup quota of {quota} CPUs; "
                      f"profiles/r06_cpu_threads_probe.txt): {med:.3f} s/step (port vs the "
                      f"reference's own CPU step: profiles/r06_cpu_ref_compare.json)"}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(nproc, argv):
    """`bench.py --gpus N` (N > 1) started without WORLD_SIZE: this parent never touches the
    GPU (it does not import the package, query devices or create a stream).  It starts N
    fresh child processes of this same script (no exec), each with RANK = LOCAL_RANK = i,
    WORLD_SIZE = N, LOCAL_WORLD_SIZE = N and MASTER_ADDR / MASTER_PORT on 127.0.0.1 -- the
    environment `torch.distributed.run --nnodes 1 --nproc-per-node N` gives, replacing the
    reference's single-device Lightning Trainer (scripts/train.py:33-43, devices=1).  Rank 0's
    stdout is the bench line; every other rank's stdout goes to stderr.  When a rank exits
    non-zero the others are terminated (by their own PIDs) and the parent exits with that
    rank's status; it returns 0 only when all N ranks returned 0."""
    import signal
    import subprocess
    port = int(os.environ.get("MASTER_PORT") or _free_port())
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nproc),
                    "LOCAL_WORLD_SIZE": str(nproc), "GROUP_RANK": "0",
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env, stdout=None if r == 0 else sys.stderr))
    status = 0
    live = list(range(nproc))
    while live:
        for r in list(live):
            rc = procs[r].poll()
            if rc is None:
                continue
            live.remove(r)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                print(f"bench launcher: rank {r} exited with {rc}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for o in live:
                    try:
                        procs[o].send_signal(signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        time.sleep(0.05)
        if status and live:  # give them 30 s to leave, then SIGKILL the stragglers
            deadline = time.time() + 30
            while time.time() < deadline and any(procs[o].poll() is None for o in live):
                time.sleep(0.1)
            for o in live:
                if procs[o].poll() is None:
                    procs[o].kill()
                    procs[o].wait()
            live = []
    return status


def dry_launch(args):
    """--dry-launch: the process-group half of the N-rank path without a model (the launcher
    test): every rank joins the group, checks the world size against --gpus, and the ranks
    exchange their ids with one all-reduce; rank 0 prints one JSON line.  --dry-fail-rank R
    makes rank R exit 3 after joining (the launcher must then exit non-zero)."""
    backend = os.environ.get("TVQ_BENCH_BACKEND", "nccl")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend)
    assert dist.get_world_size() == args.gpus == world, (dist.get_world_size(), args.gpus)
    if args.dry_fail_rank == rank:
        print(f"rank {rank}: forced failure (--dry-fail-rank)", file=sys.stderr, flush=True)
        os._exit(3)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else "cpu"
    ids = torch.zeros(world, dtype=torch.int64, device=dev)
    ids[rank] = rank + 1
    dist.all_reduce(ids)
    if rank == 0:
        print(json.dumps({"dry_launch": True, "world_size": dist.get_world_size(),
                          "backend": dist.get_backend(), "ranks": [int(v) - 1 for v in ids]}),
              flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-sampler", action="store_true")
    ap.add_argument("--no-config0", action="store_true")
    ap.add_argument("--no-stage-legs", action="store_true", help="skip the per-stage legs")
    ap.add_argument("--eager", action="store_true", help="no hipGraph capture of the step")
    ap.add_argument("--dry-launch", action="store_true",
                    help="launcher check: join the process group, exchange rank ids, no model")
    ap.add_argument("--dry-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args.gpus, sys.argv[1:]))
    if args.dry_launch:
        return dry_launch(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N ranks "
                         f"with `python bench.py --gpus N` or torch.distributed.run "
                         f"--nproc-per-node N ... bench.py --gpus N")
    # rehearsal of the N > 1 path on a one-GPU box (all ranks on cuda:0 over gloo; RCCL
    # refuses two ranks on one device): TVQ_BENCH_REHEARSAL=1.  Timings so obtained are not
    # scaling numbers.
    rehearsal = os.environ.get("TVQ_BENCH_REHEARSAL", "0") == "1"
    if rehearsal:
        local = 0
    if world > 1:
        if not rehearsal and torch.cuda.device_count() < world:
            raise SystemExit(f"bench.py: {world} ranks but {torch.cuda.device_count()} visible GPUs")
        torch.cuda.set_device(local)
        dist.init_process_group("gloo" if rehearsal else "nccl")
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
        assert rehearsal or dist.get_backend() == "nccl", dist.get_backend()
    device = torch.device("cuda", local)
    tr = JointTrainer(device, world)
    batch = synthetic_batch(1234 + rank, device)
    if not args.eager:
        tr.capture(batch)

    for _ in range(args.warmup):
        tr.step(batch)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out1, out2 = tr.step(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rank_elapsed = [elapsed]
    if world > 1:
        t = torch.zeros(world, device=device, dtype=torch.float64)
        t[rank] = elapsed
        dist.all_reduce(t, op=dist.ReduceOp.SUM)  # every rank's own elapsed time
        rank_elapsed = [float(v) for v in t.cpu()]
        elapsed = max(rank_elapsed)
    loss1 = float(out1["loss"].detach().sum())
    loss2 = float(out2["loss"].detach())

    if rank == 0:
        value = world * args.steps / elapsed
        res = {
            "metric": "stage1+stage2 train steps/sec on synthetic (B,C,T) trajectories, 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic",
            "config": {"workload": "stage1 VQ-VAE + stage2 MaskGIT joint train step, per-GPU batch "
                                   "(B=256,C=6,T=256), K=512, configs/config.yaml architecture",
                       "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world}",
                       "launch": "eager" if args.eager else "hipgraph",
                       "value_counts": "per-GPU B=256 joint steps summed over the ranks (one "
                                       "optimizer step per N of them at N>1)",
                       "optimizer_steps_per_s": round(args.steps / elapsed, 3),
                       "trajectories_per_s": round(value * B, 1)},
            "losses": {"stage1": round(loss1, 5), "stage2": round(loss2, 5)},
            "peak_mem_gb": round(torch.cuda.max_memory_allocated(device) / 2 ** 30, 3),
        }
        if world > 1:
            res["dist"] = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                           "rank_elapsed_s": [round(v, 6) for v in rank_elapsed],
                           "physical_gpus": 1 if rehearsal else world}
            if rehearsal:
                res["rehearsal"] = True
                res["parallelism_note"] = ("REHEARSAL: every rank on cuda:0 over gloo; not a "
                                           "multi-GPU measurement")
        if not args.no_roofline:
            res["roofline"] = roofline_leg(device, res["ms_per_step"])
        if not args.no_config0 and world == 1:  # (before the sampler: rank 0 only)
            res["config0"] = config0_leg(device, cpu=not args.no_cpu_baseline)
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline_leg()
    if not args.no_sampler:  # every rank: replicas sample concurrently at world > 1
        samp = sampler_leg(tr, device, world=world)
    # each stage's optimizer step alone (graph-replayed; the reference trains them one after
    # the other), beside the concurrent joint step -- last, since its extra optimizer steps
    # move the weights, LR schedule, BN statistics and codebooks the sampler leg reads
    alone = None
    if world == 1 and not args.eager and not args.no_stage_legs:
        alone = {w: round(tr.stage_alone_ms(batch, w), 3) for w in ("stage1", "stage2")}
    if rank == 0:
        if not args.no_sampler:
            res["sampler"] = samp
        if alone is not None:
            res["stage1_ms_per_step"] = alone["stage1"]
            res["stage2_ms_per_step"] = alone["stage2"]
            res["sequential_ms_per_step"] = round(alone["stage1"] + alone["stage2"], 3)
            res["ms_per_step_is"] = ("stage1 and stage2 steps run concurrently on one GPU "
                                     "(independent: stage2 trains on a frozen stage1 snapshot); "
                                     "sequential_ms_per_step = the two stages alone, one after "
                                     "the other, as the reference trains them")
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
