"""Data-parallel logic on CPU (gloo, world_size 2): the pieces of the multi-GPU step that
are not kernels -- the flat-gradient all-reduce/average of bench.JointTrainer and the
deferred sync_codebook reduction of hip.vq.CodebookUpdate (the reference's
sync_codebook all-reduce of cluster sizes and embedding sums, vq.py:229,234).  The DP
step exchanges each stage's gradients and BatchNorm statistics separately (right after
that stage's backward); that split exchange is checked bitwise equal to one flat
exchange of everything."""
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

        # flat gradient average (JointTrainer._allreduce -> hip.dp.ReplicaSync) over the
        # real stage1 / stage2 parameter count, + layer-dropout gates OR-ed over ranks (a
        # segment some replica used is updated on every replica)
        import copy
        from timevqvae.hip.dp import ReplicaSync, batchnorm_modules, flatten_bn_buffers
        from timevqvae.trainers import Stage1, Stage2
        from timevqvae.utils import set_seed
        set_seed(0)  # identical initial replicas (bench.JointTrainer also broadcasts rank 0's)
        cfg = bench.config(True)
        s1 = Stage1(64, 3, cfg)
        s2 = Stage2(None, None, 64, 3, bench.N_CLASSES, config=cfg, stage1=copy.deepcopy(s1))
        nparam = sum(p.numel() for p in s1.parameters())
        g = torch.Generator().manual_seed(100 + rank)

        class Opt:
            flat_grad = torch.randn(nparam, generator=g)
            has_gates = True
            gates = torch.tensor([1.0, 0.0, 0.0]) if rank == 0 else torch.tensor([0.0, 0.0, 1.0])
        tr = bench.JointTrainer.__new__(bench.JointTrainer)
        tr.world = world
        tr.sync = ReplicaSync(world)
        opt = Opt()
        mine = opt.flat_grad.clone()
        both = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(both, mine)
        tr._allreduce(opt)
        ok_grad = torch.allclose(opt.flat_grad, sum(both) / world, rtol=1e-6, atol=1e-7)
        ok_grad = ok_grad and torch.equal(opt.gates, torch.tensor([1.0, 0.0, 1.0]))

        # BatchNorm running statistics: one flat buffer (every running_mean / running_var
        # a view of it), averaged over the replicas -> every state_dict tensor bitwise
        # equal across ranks (DDP broadcast_buffers semantics)
        mods = [s1, s2.maskgit.transformer_l, s2.maskgit.transformer_h]
        # one flat buffer per stage, as JointTrainer holds them
        tr.bn_flat = [flatten_bn_buffers([s1]), flatten_bn_buffers(mods[1:])]
        bns = batchnorm_modules(mods)
        with torch.no_grad():  # per-rank updates, as each replica's forward makes them
            for b in bns:
                b.running_mean.add_(torch.randn(b.running_mean.shape, generator=g))
                b.running_var.mul_(1 + torch.rand(b.running_var.shape, generator=g))
        views_ok = all(any(f.data_ptr() <= b.running_mean.data_ptr() < f.data_ptr() +
                           4 * f.numel() for f in tr.bn_flat) for b in bns)
        pre = torch.cat([torch.cat([b.running_mean, b.running_var]) for b in bns])
        # the DP form's split exchange (each stage's buffer right after its backward) is
        # bitwise equal to one flat exchange of everything
        flat_once = torch.cat([f.clone() for f in tr.bn_flat])
        ReplicaSync(world).buffers(flat_once)
        tr._sync_buffers((0,))
        tr._sync_buffers((1,))
        ok_split = torch.equal(torch.cat(tr.bn_flat), flat_once)
        sd = {k: v.clone() for m in (s1, s2) for k, v in m.state_dict().items()}
        gathered = [None] * world
        dist.all_gather_object(gathered, sd)
        ok_sd = all(torch.equal(gathered[0][k], gathered[r][k]) for r in range(world)
                    for k in sd)
        pres = [torch.empty_like(pre) for _ in range(world)]
        dist.all_gather(pres, pre)
        post = torch.cat([torch.cat([b.running_mean, b.running_var]) for b in bns])
        ok_bn = views_ok and ok_sd and ok_split and torch.allclose(post, sum(pres) / world,
                                                                   rtol=1e-6, atol=1e-6)
        # the same for the flat gradients: stage1's and stage2's buffers exchanged
        # separately == one exchange of their concatenation, bitwise
        g1 = torch.randn(nparam, generator=g)
        g2 = torch.randn(sum(p.numel() for p in s2.parameters() if p.requires_grad),
                         generator=g)

        class O:
            def __init__(self, t):
                self.flat_grad, self.has_gates = t, False
        both_once = O(torch.cat([g1, g2]))
        o1, o2 = O(g1.clone()), O(g2.clone())
        tr._allreduce(both_once)
        tr._allreduce(o1)
        tr._allreduce(o2)
        ok_bn = ok_bn and torch.equal(torch.cat([o1.flat_grad, o2.flat_grad]), both_once.flat_grad)
        ok_grad = ok_grad and ok_bn

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
