"""The data-parallel step on the GPU: two processes on cuda:0 (gloo), each holding its own
shard of the batch, run bench.JointTrainer(world=2) through capture() -- the hipGraph path
with the codebook updates deferred between the two graph segments, where the flat-gradient
average and the sync_codebook all-reduce of the per-code statistics run (reference
vq.py:155,229,234: every replica's EMA sees the global batch).

Two DP forms: the default overlaps each stage's exchange with the other stage's backward
(separate graphs per stage); TVQ_DP_OVERLAP=0 runs every exchange after one fwd+bwd graph.
Checked after each of 3 replayed steps:
  * the flat stage1 / stage2 parameters, the stage1 codebook buffers and every other
    state_dict tensor (BatchNorm running statistics included) are bitwise equal across
    the ranks (replicas never drift);
  * the stage1 codebook EMA (cluster_size, embed_avg, embed) equals the oracle
    vq_ref.ema over the CONCATENATED shards -- the rank-0 and rank-1 VQ inputs and
    assignments of that step -- from the pre-step buffers."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS = 3


def _worker(rank, world, port, out_dir, overlap):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TVQ_DP_OVERLAP=overlap)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = bench.JointTrainer(dev, world)
    batch = bench.synthetic_batch(1234 + rank, dev)
    vqs = {"l": tr.s1.vq_model_l, "h": tr.s1.vq_model_h}
    seen = {}

    def hook(band):
        def f(mod, args, out):
            # graph-pool tensors: held here, so after every replay they hold that replay's
            # VQ input (B, N, D) and assignment (B, N)
            seen[band] = (args[0], out[1])
        return f
    for band, m in vqs.items():
        m.register_forward_hook(hook(band))
    tr.capture(batch)
    graph_kind = type(tr.graph).__name__
    bufs = lambda m: {k: getattr(m._codebook, k).detach().cpu().clone()  # noqa: E731
                      for k in ("cluster_size", "embed_avg", "embed")}
    log = []
    for _ in range(STEPS):
        pre = {b: bufs(m) for b, m in vqs.items()}
        out1, out2 = tr.step(batch)
        torch.cuda.synchronize()
        rec = {"pre": pre, "post": {b: bufs(m) for b, m in vqs.items()},
               "x": {b: seen[b][0].detach().reshape(-1, seen[b][0].shape[-1]).cpu().clone()
                     for b in vqs},
               "idx": {b: seen[b][1].detach().reshape(-1).cpu().clone() for b in vqs},
               "flat1": tr.opt1.flat.detach().cpu().clone(),
               "flat2": tr.opt2.flat.detach().cpu().clone(),
               "loss1": float(out1["loss"].detach().sum()), "loss2": float(out2["loss"].detach()),
               "graph": graph_kind,
               "state": {f"s{i}.{k}": v.detach().cpu().clone()
                         for i, m in ((1, tr.s1), (2, tr.s2)) for k, v in m.state_dict().items()}}
        log.append(rec)
    torch.save(log, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


_runs = {}


def _run(overlap, tmp_path_factory):
    """Both ranks' logs of a 3-step world-2 run in one DP form (cached per module)."""
    if overlap not in _runs:
        d = tmp_path_factory.mktemp(f"dp{overlap}")
        ctx = mp.get_context("spawn")
        port = 29500 + (os.getpid() % 500) + 10 * int(overlap)
        procs = [ctx.Process(target=_worker, args=(r, 2, port, str(d), overlap))
                 for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=100)
        for p in procs:
            if p.is_alive():
                p.kill()
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        _runs[overlap] = (torch.load(d / "rank0.pt", weights_only=True),
                          torch.load(d / "rank1.pt", weights_only=True))
    return _runs[overlap]


@pytest.mark.gpu
def test_joint_trainer_world2_graph_path(tmp_path_factory):
    """The default DP form: stage1 / stage2 as two graphs on two streams, each stage's
    exchange issued right after its backward (hip.graph.BranchStepGraph)."""
    r0, r1 = _run("1", tmp_path_factory)
    assert r0[0]["graph"] == "BranchStepGraph"
    from oracle import vq_ref
    for s, (a, b) in enumerate(zip(r0, r1)):
        assert np.isfinite(a["loss1"]) and np.isfinite(a["loss2"])
        assert torch.equal(a["flat1"], b["flat1"]), f"step {s}: stage1 replicas differ"
        assert torch.equal(a["flat2"], b["flat2"]), f"step {s}: stage2 replicas differ"
        # every state_dict tensor (parameters, BatchNorm running statistics, codebooks,
        # counters) bitwise equal across the replicas (DDP broadcast_buffers semantics)
        assert a["state"].keys() == b["state"].keys()
        diff = [k for k in a["state"] if not torch.equal(a["state"][k], b["state"][k])]
        assert not diff, f"step {s}: state_dict entries differ across ranks: {diff[:5]}"
        if s == 0:
            assert not torch.equal(a["flat1"], torch.zeros_like(a["flat1"]))
            rm = [k for k in a["state"] if k.startswith("s1.") and k.endswith("running_mean")]
            assert rm and any(a["state"][k].abs().sum() > 0 for k in rm)  # BN stats moved
        for band in ("l", "h"):
            for k in ("cluster_size", "embed_avg", "embed"):
                assert torch.equal(a["post"][band][k], b["post"][band][k]), (s, band, k)
                assert torch.equal(a["pre"][band][k], b["pre"][band][k]), (s, band, k)
            # the shards are different data
            assert not torch.equal(a["x"][band], b["x"][band])
            x = torch.cat([a["x"][band], b["x"][band]]).numpy().astype(np.float32)
            idx = torch.cat([a["idx"][band], b["idx"][band]]).numpy().astype(np.int64)
            pre = a["pre"][band]
            cs, ea, E, counts, _ = vq_ref.ema(x, idx, pre["cluster_size"].numpy(),
                                             pre["embed_avg"].numpy())
            assert counts.sum() == x.shape[0]
            post = a["post"][band]
            np.testing.assert_allclose(post["cluster_size"].numpy(), cs, rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(post["embed_avg"].numpy(), ea, rtol=1e-5, atol=1e-4)
            np.testing.assert_allclose(post["embed"].numpy(), E, rtol=1e-4, atol=1e-4)
            # and not the single-shard EMA: the sync actually happened
            cs_1, _, _, _, _ = vq_ref.ema(a["x"][band].numpy(), a["idx"][band].numpy(),
                                          pre["cluster_size"].numpy(), pre["embed_avg"].numpy())
            assert not np.allclose(cs_1, cs)
    # the replicas moved (3 optimizer steps)
    assert not torch.equal(r0[0]["flat1"], r0[-1]["flat1"])


@pytest.mark.gpu
def test_dp_overlap_equals_two_segment_form(tmp_path_factory):
    """The overlapped form (each stage exchanged after its own backward, separate graphs)
    and the two-segment form (TVQ_DP_OVERLAP=0: one fwd+bwd graph, every exchange after
    it) give bitwise-equal replicas after every step: same kernels, same dropout draws, the
    split exchange is elementwise the flat one."""
    a0, _ = _run("1", tmp_path_factory)
    b0, _ = _run("0", tmp_path_factory)
    assert b0[0]["graph"] == "StepGraph"
    for s, (a, b) in enumerate(zip(a0, b0)):
        assert torch.equal(a["flat1"], b["flat1"]), f"step {s}: stage1 differs"
        assert torch.equal(a["flat2"], b["flat2"]), f"step {s}: stage2 differs"
        diff = [k for k in a["state"] if not torch.equal(a["state"][k], b["state"][k])]
        assert not diff, f"step {s}: {diff[:5]}"
