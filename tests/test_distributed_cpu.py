"""World-size-2 gloo test of the data-parallel path (CPU metric mode): sharded scores
all-gathered across ranks equal the single-process result."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fast_speech_enhancement_metrics_amd import PESQ, STOI
        from fast_speech_enhancement_metrics_amd.distributed import sharded_scores
        from tests.conftest import load_golden
        g = load_golden("pesq_wide")
        p = sharded_scores(PESQ(16000), torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"]))
        gs = load_golden("stoi_wide")
        s = sharded_scores(STOI(16000), torch.from_numpy(gs["clean_f"]), torch.from_numpy(gs["noisy_f"]))
        out_q.put((rank, p.numpy(), s.numpy()))
    finally:
        dist.destroy_process_group()


def test_sharded_gather_matches_single_process():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    from tests.conftest import load_golden
    g = load_golden("pesq_wide")
    ref_p = PESQ(16000).scores(torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"])).numpy()
    gs = load_golden("stoi_wide")
    ref_s = torch.stack(STOI(16000).scores(torch.from_numpy(gs["clean_f"]), torch.from_numpy(gs["noisy_f"]),
                                           sample_rate=16000), 1).numpy()
    for rank, p, s in res:
        np.testing.assert_allclose(p[:, 0], ref_p, rtol=0, atol=1e-6)
        np.testing.assert_allclose(s, ref_s, rtol=0, atol=1e-6)


@pytest.mark.parametrize("batch,world", [(7, 2), (8, 4), (3, 8), (4096, 8)])
def test_shard_bounds_cover_batch(batch, world):
    from fast_speech_enhancement_metrics_amd.distributed import shard_bounds
    b = [shard_bounds(batch, world, r) for r in range(world)]
    assert b[0][0] == 0 and b[-1][1] == batch
    assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
    sizes = [hi - lo for lo, hi in b]
    assert max(sizes) - min(sizes) <= 1


def _worker_ragged(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fast_speech_enhancement_metrics_amd import PESQ, STOI
        from fast_speech_enhancement_metrics_amd.distributed import sharded_scores_ragged
        from tests.conftest import load_golden
        g = load_golden("varlen_16k")
        cl = [torch.from_numpy(g["clean_f"][b, :n]) for b, n in enumerate(g["lengths"])]
        dl = [torch.from_numpy(g["noisy_f"][b, :n]) for b, n in enumerate(g["lengths"])]
        p = sharded_scores_ragged(PESQ(16000), cl, dl)
        s = sharded_scores_ragged(STOI(16000), cl, dl)
        out_q.put((rank, p.numpy(), s.numpy()))
    finally:
        dist.destroy_process_group()


def test_ragged_lpt_sharding_matches_reference():
    """Config-5 style ragged batch over 2 gloo ranks (LPT by total length) == golden."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker_ragged, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from tests.conftest import load_golden
    g = load_golden("varlen_16k")
    for rank, p, s in res:
        for got, want, tol in ((p[:, 0], g["pesq"], 2e-3), (s[:, 0], g["stoi"], 1e-4), (s[:, 1], g["estoi"], 1e-4)):
            assert np.array_equal(np.isnan(got), np.isnan(want))
            m = ~np.isnan(want)
            np.testing.assert_allclose(got[m], want[m], atol=tol, rtol=0)


def test_lpt_shards_balance():
    from fast_speech_enhancement_metrics_amd.distributed import lpt_shards
    rng = np.random.default_rng(0)
    lens = rng.integers(32000, 480000, size=1000)
    plan = lpt_shards(lens, 8)
    assert sorted(i for s in plan for i in s) == list(range(1000))
    loads = [int(lens[s].sum()) for s in plan]
    assert max(loads) - min(loads) <= lens.max()  # LPT bound
    assert (max(loads) - min(loads)) / np.mean(loads) < 0.01


def _spawn(target, world, *args):
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _worker_rates(rank, world, port, out_q):
    """Metrics configured for 8 kHz score 8 kHz rows: the helpers pass metric.sample_rate."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI
        from fast_speech_enhancement_metrics_amd.distributed import sharded_scores, sharded_scores_ragged
        from tests.conftest import load_golden
        g = load_golden("rate_8k")
        c, n = torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"])
        p = sharded_scores(PESQ(8000), c, n)
        s = sharded_scores(STOI(8000), c, n)
        j = sharded_scores(PESQ_STOI(8000), c, n)
        pr = sharded_scores_ragged(PESQ(8000), list(c), list(n))
        out_q.put((rank, p.numpy(), s.numpy(), j.numpy(), pr.numpy()))
    finally:
        dist.destroy_process_group()


def test_sharded_scores_use_metric_rate():
    """PESQ(8000) / STOI(8000) / PESQ_STOI(8000) over 2 gloo ranks == the reference's 8 kHz golden
    (before, scores() treated the 8 kHz rows as 16 kHz / 10 kHz rows)."""
    from tests.conftest import load_golden
    g = load_golden("rate_8k")
    for rank, p, s, j, pr in _spawn(_worker_rates, 2):
        np.testing.assert_allclose(p[:, 0], g["pesq"], atol=2e-3, rtol=0)
        np.testing.assert_allclose(pr[:, 0], g["pesq"], atol=2e-3, rtol=0)
        np.testing.assert_allclose(s[:, 0], g["stoi"], atol=1e-4, rtol=0)
        np.testing.assert_allclose(s[:, 1], g["estoi"], atol=1e-4, rtol=0)
        np.testing.assert_allclose(j, np.stack([g["pesq"], g["stoi"], g["estoi"]], 1), atol=2e-3, rtol=0)


def test_scores_without_rate_refuse_other_rates():
    from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI
    x = torch.zeros(1, 16000)
    for m in (PESQ(8000), STOI(16000), PESQ_STOI(8000)):
        with pytest.raises(ValueError, match="sample_rate"):
            m.scores(x, x)


def _worker_empty(rank, world, port, out_q):
    """Batches smaller than the world: ranks with no rows still join the all-gather."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fast_speech_enhancement_metrics_amd import PESQ, STOI
        from fast_speech_enhancement_metrics_amd.distributed import sharded_scores, sharded_scores_ragged
        from tests.conftest import load_golden
        g = load_golden("pesq_wide")
        c, n = torch.from_numpy(g["clean_f"][:1]), torch.from_numpy(g["noisy_f"][:1])
        p = sharded_scores(PESQ(16000), c, n)
        s = sharded_scores(STOI(16000), c, n)
        pr = sharded_scores_ragged(PESQ(16000), list(c), list(n))
        out_q.put((rank, p.numpy(), s.numpy(), pr.numpy()))
    finally:
        dist.destroy_process_group()


def test_empty_shards():
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    from tests.conftest import load_golden
    g = load_golden("pesq_wide")
    c, n = torch.from_numpy(g["clean_f"][:1]), torch.from_numpy(g["noisy_f"][:1])
    ref_p = PESQ(16000).scores(c, n).numpy()
    ref_s = torch.stack(STOI(16000).scores(c, n, sample_rate=16000), 1).numpy()
    for rank, p, s, pr in _spawn(_worker_empty, 3):
        assert p.shape == (1, 1) and s.shape == (1, 2) and pr.shape == (1, 1)
        np.testing.assert_allclose(p[:, 0], ref_p, atol=1e-6, rtol=0)
        np.testing.assert_allclose(pr[:, 0], ref_p, atol=1e-6, rtol=0)
        np.testing.assert_allclose(s, ref_s, atol=1e-6, rtol=0)


def _scatter_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fast_speech_enhancement_metrics_amd import PESQ_STOI
        from fast_speech_enhancement_metrics_amd.distributed import scatter_batch, sharded_scores_from
        from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
        src = 1
        c = n = lens = None
        if rank == src:  # only the source rank holds the batch
            c, n, _ = speech_like_pairs(5, 24000, 16000, seed=3)
            lens = torch.tensor([24000, 20000, 24000, 9000, 16001], dtype=torch.int32)
        cs, ns, ls, B = scatter_batch(c, n, src=src, lengths=lens)
        s = sharded_scores_from(PESQ_STOI(16000), c, n, src=src, lengths=lens)
        out_q.put((rank, B, cs.numpy(), ns.numpy(), ls.numpy(), s.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_scatter_from_one_rank(world):
    """Inputs held by one rank: each rank receives exactly its shard_bounds rows and
    lengths, and the scattered, sharded, gathered scores equal the single-process result."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    from fast_speech_enhancement_metrics_amd.distributed import shard_bounds
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(5, 24000, 16000, seed=3)
    lens = torch.tensor([24000, 20000, 24000, 9000, 16001], dtype=torch.int32)
    ref = torch.stack(PESQ_STOI(16000).scores(c, n, lengths=lens), 1).numpy()
    for rank, B, cs, ns, ls, s in res:
        lo, hi = shard_bounds(5, world, rank)
        assert B == 5
        np.testing.assert_array_equal(cs, c[lo:hi].numpy())
        np.testing.assert_array_equal(ns, n[lo:hi].numpy())
        np.testing.assert_array_equal(ls, lens[lo:hi].numpy())
        np.testing.assert_allclose(s, ref, rtol=0, atol=1e-6, equal_nan=True)


def _scatter_bad_worker(rank, world, port, out_q):
    """scatter_batch with (a) clean float64 / noisy float32, (b) int16 codes, (c) mismatched
    shapes on the source: (a) and (b) arrive as float32 rows on every rank, (c) raises on EVERY
    rank (no rank left blocked in a collective)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fast_speech_enhancement_metrics_amd.distributed import scatter_batch
        from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs, to_int16
        c, n, _ = speech_like_pairs(3, 4000, 16000, seed=4)
        res = {}
        a = scatter_batch(c.double() if rank == 0 else None, n if rank == 0 else None, src=0)
        res["mixed"] = (a[0].dtype, a[1].dtype, a[0].numpy(), a[1].numpy())
        b = scatter_batch(to_int16(c) if rank == 0 else None, to_int16(n) if rank == 0 else None, src=0)
        res["int16"] = (b[0].dtype, b[0].numpy())
        try:
            scatter_batch(c[:, :100] if rank == 0 else None, n if rank == 0 else None, src=0)
            res["bad"] = None
        except ValueError as e:
            res["bad"] = str(e)
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_scatter_mixed_dtypes_and_bad_shapes():
    from fast_speech_enhancement_metrics_amd.distributed import shard_bounds
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs, to_int16
    c, n, _ = speech_like_pairs(3, 4000, 16000, seed=4)
    for rank, res in _spawn(_scatter_bad_worker, 2):
        lo, hi = shard_bounds(3, 2, rank)
        dc, dn, rc, rn = res["mixed"]
        assert dc == torch.float32 and dn == torch.float32
        np.testing.assert_array_equal(rc, c[lo:hi].double().float().numpy())
        np.testing.assert_array_equal(rn, n[lo:hi].numpy())
        d16, r16 = res["int16"]
        assert d16 == torch.float32
        np.testing.assert_array_equal(r16, to_int16(c)[lo:hi].float().numpy())
        assert res["bad"] is not None and "one shape" in res["bad"]
