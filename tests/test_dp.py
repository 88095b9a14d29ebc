"""Data-parallel logic on CPU (gloo, world_size 2): the pieces of the multi-GPU step that
are not kernels -- the flat-gradient all-reduce/average of bench.JointTrainer and the
deferred sync_codebook reduction of hip.vq.CodebookUpdate (the reference's
sync_codebook all-reduce of cluster sizes and embedding sums, vq.py:229,234)."""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import bench
        from timevqvae.hip.vq import CodebookUpdate

        # flat gradient average (JointTrainer._allreduce)
        # + layer-dropout gates OR-ed over ranks (a segment some replica used is updated
        # on every replica)
        class Opt:
            flat_grad = torch.full((5,), float(rank + 1))
            has_gates = True
            gates = torch.tensor([1.0, 0.0, 0.0]) if rank == 0 else torch.tensor([0.0, 0.0, 1.0])
        tr = bench.JointTrainer.__new__(bench.JointTrainer)
        tr.world = world
        opt = Opt()
        tr._allreduce(opt)
        ok_grad = torch.allclose(opt.flat_grad, torch.full((5,), (1 + world) / 2.0))
        ok_grad = ok_grad and torch.equal(opt.gates, torch.tensor([1.0, 0.0, 1.0]))

        # sync_codebook statistics: summed over ranks before the EMA
        K, D = 4, 3
        cs = torch.arange(K, dtype=torch.float32) + rank
        es = torch.ones(K, D) * (rank + 1)
        emb = torch.zeros(K, D)
        u = CodebookUpdate(cs, es, torch.zeros(K), torch.zeros(K, D), emb, 0.8, 1e-5,
                           lambda t: dist.all_reduce(t))
        u.reduce()
        ok_cs = torch.equal(cs, 2 * torch.arange(K, dtype=torch.float32) + 1)
        ok_es = torch.equal(es, torch.full((K, D), 3.0))
        q.put((rank, ok_grad, ok_cs, ok_es))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), None, None))


def test_dp_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29000 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1:] == (True, True, True), r
