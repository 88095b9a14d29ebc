"""The deterministic group-by sums behind nn.Embedding's backward and the VQ embed_sum
(csrc/tvq_reduce.hip: gb_sort1_kernel -- the single-block stable counting sort -- or the
3-launch sort above 2048 rows, then seg_sum_kernel with its in-launch combine of skewed
values) against torch fp64 index_add, on uniform, skewed (one value owning 60 % of the rows,
as the MaskGIT mask token does), sparse (most values empty) and tiny (the class embedding)
index sets, and a 5000-value vocabulary (the wide placement kernel); every call is run
twice and must be bitwise equal.  Tolerance: rel-L2 1e-6
against fp64 (fp32 sums of <= 32768 rows in a fixed order)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(kind, M, V, gen):
    if kind == "uniform":
        return torch.randint(0, V, (M,), generator=gen)
    if kind == "skewed":
        idx = torch.randint(0, V, (M,), generator=gen)
        hot = torch.rand(M, generator=gen) < 0.6
        return torch.where(hot, torch.full_like(idx, V - 1), idx)
    if kind == "sparse":
        return torch.randint(0, 7, (M,), generator=gen) * (V // 7)
    if kind == "invalid":  # out-of-range indices (-1, V + 3) are skipped by the group-by
        idx = torch.randint(0, V, (M,), generator=gen)
        bad = torch.rand(M, generator=gen)
        idx = torch.where(bad < 0.05, torch.full_like(idx, -1), idx)
        return torch.where(bad > 0.95, torch.full_like(idx, V + 3), idx)
    raise ValueError(kind)


@pytest.mark.parametrize("kind,M,V,D", [
    ("uniform", 24576, 513, 128), ("skewed", 24576, 513, 128), ("sparse", 6144, 513, 128),
    ("uniform", 256, 6, 256), ("skewed", 6144, 513, 64), ("uniform", 32768, 1024, 32),
    ("skewed", 40000, 300, 128), ("uniform", 3, 1, 128), ("skewed", 8192, 5000, 32),
    # the single-block sort at its largest LDS footprint (M = 2048, V = 1024: ~68 KB), skewed,
    # and out-of-range indices on both paths
    ("skewed", 2048, 1024, 128), ("uniform", 2048, 1000, 64), ("invalid", 2048, 1024, 64),
    ("invalid", 6144, 513, 128)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_embedding_bwd_groupby(kind, M, V, D, accumulate, cuda):
    from timevqvae.hip._native import call, plan_trace, ptr, stream_ptr, value
    gen = torch.Generator().manual_seed(M + V + D)
    idx = _case(kind, M, V, gen)
    g = torch.randn(M, D, generator=gen)
    t0 = torch.randn(V, D, generator=gen)
    ref = t0.double() * accumulate
    ok = (idx >= 0) & (idx < V)
    ref = ref.index_add(0, idx[ok], g[ok].double())
    idd, gd = idx.to(cuda), g.to(cuda)
    outs = []
    for _ in range(2):
        tg = t0.to(cuda)
        ws = torch.empty(value("tvq_embedding_bwd_workspace", M, V), device=cuda, dtype=torch.int32)
        with plan_trace() as tr:
            call("tvq_embedding_bwd", ptr(idd), M, D, ptr(gd), D, V, ptr(tg), int(accumulate), -1,
                 0.0, None, 0, ptr(ws), stream_ptr())
            torch.cuda.synchronize()
        outs.append(tg.cpu())
    assert torch.equal(outs[0], outs[1])
    want = "group_by sort1" if M <= 2048 and V <= 1024 else "group_by 3-launch"
    assert tr.has(want), tr.lines
    err = float((outs[0].double() - ref).norm() / ref.norm())
    assert err < 1e-6, err


def test_vq_stats_groupby_full_size(cuda):
    """tvq_vq_stats at the HF band's training shape (24576 token rows of the (256,128,3,32)
    latent, K = 512) with a collapsed code: counts exact, embed_sum within 1e-6 of fp64."""
    from timevqvae.hip._native import call, ptr, stream_ptr, value
    gen = torch.Generator().manual_seed(9)
    B, D, N, K = 256, 128, 96, 512
    M = B * N
    x = torch.randn(B, D, N, generator=gen)
    idx = _case("skewed", M, K, gen).to(torch.int32)
    xt = x.permute(0, 2, 1).reshape(M, D)
    ref = torch.zeros(K, D, dtype=torch.float64).index_add(0, idx.long(), xt.double())
    xd, idd = x.to(cuda), idx.to(cuda)
    counts = torch.empty(K, dtype=torch.int32, device=cuda)
    cs = torch.empty(K, device=cuda)
    es = torch.empty(K, D, device=cuda)
    ws = torch.empty(value("tvq_vq_stats_workspace", M, K), dtype=torch.int32, device=cuda)
    call("tvq_vq_stats", ptr(xd), B, N, D, D * N, 1, N, ptr(idd), K, ptr(counts), ptr(cs), ptr(es),
         ptr(ws), stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(counts.cpu(), torch.bincount(idx.long(), minlength=K).to(torch.int32))
    assert torch.equal(cs.cpu(), counts.cpu().float())
    err = float((es.cpu().double() - ref).norm() / ref.norm())
    assert err < 1e-6, err
