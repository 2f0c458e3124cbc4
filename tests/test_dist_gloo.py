"""Data-parallel harness (qnn/dist.py) on CPU with the gloo backend, world_size 2.

The GPU path is the same code with backend "nccl" (RCCL); only the collective's
transport differs.  Checks: contiguous ragged sharding, gather-to-root equals
the unsharded forward, non-root ranks get None, batch independence; the asynchronous
double-buffered gather over a static-buffer engine through bench.py's timed region;
the bucketed all-reduce of calibrated ranges.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from qnn.dist import ShardedInference, shard_bounds


def test_shard_bounds_cover_batch_exactly():
    for gb in (1, 7, 128, 2048, 1001):
        for world in (1, 2, 3, 4, 8):
            spans = [shard_bounds(gb, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == gb
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, gb, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 10), torch.nn.ReLU(), torch.nn.Linear(10, 5)).eval()
    x_all = torch.randn(gb, 16, generator=torch.Generator().manual_seed(42))
    runner = ShardedInference(model, gb)
    s, e = runner.local_slice()
    out = runner(x_all[s:e])
    if rank == 0:
        with torch.no_grad():
            ref = model(x_all)
        q.put(("root", out.shape == ref.shape and bool(torch.allclose(out, ref, rtol=0, atol=1e-6))))
    else:
        q.put(("other", out is None))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("gb", [8, 7, 129])
def test_gather_matches_unsharded_world2(gb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, gb, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(2))
    assert res == {"root": True, "other": True}


class _StaticEngine:
    """Stands in for qnn.Engine on CPU: planned for exactly N samples, returns its static
    logits buffer (the next call overwrites it), as Engine.__call__ does."""

    def __init__(self, n, w):
        self.N, self.w = n, w
        self.logits = torch.empty(n, w.shape[1])

    def __call__(self, x):
        assert x.shape[0] == self.N
        torch.matmul(x, self.w, out=self.logits)
        return self.logits


def _engine_worker(rank, world, port, gb, steps, q):
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = torch.randn(16, 5, generator=torch.Generator().manual_seed(3))
    xs = [torch.randn(gb, 16, generator=torch.Generator().manual_seed(100 + k)) for k in range(steps)]
    s, e = shard_bounds(gb, world, rank)
    eng = _StaticEngine(e - s, w)
    runner = ShardedInference(eng, gb)
    # every step in flight before any result is read: the double-buffered send slots keep
    # each step's logits although the engine's static buffer is overwritten by the next step
    handles = [runner.submit(x[s:e]) for x in xs]
    outs = [h.result() for h in handles]
    ok = all(o is None for o in outs) if rank else \
        all(torch.allclose(o, x @ w, rtol=0, atol=1e-5) for o, x in zip(outs, xs))
    # bench.py's timed region + aggregation over the same runner
    k = iter(range(10 ** 6))
    elapsed = bench.timed_run(lambda: runner.submit(xs[next(k) % steps][s:e]), steps, 1, world)
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    same = t.item() == elapsed  # MAX over ranks: every rank reports the same time
    q.put((rank, ok, same, bench.throughput(gb, steps, elapsed) == gb * steps / elapsed))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("gb", [7, 129])
def test_sharded_engine_async_gather_ragged_world2(gb):
    """ShardedInference over a static-buffer engine per rank (ragged shards 4/3 and 65/64),
    driven through bench.py's timed_run / throughput."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker, args=(r, 2, port, gb, 4, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert res == [(0, True, True, True), (1, True, True, True)]


def _calib_worker(rank, world, port, q):
    from oracle import qnn_oracle as O
    from qnn import synthetic
    from qnn.dist import allreduce_calibration
    from qnn.quantize import QConv2d, RangeBN
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = torch.nn.Sequential(QConv2d(4, 8, 3, padding=1, bias=False), RangeBN(8))

    def states(r):  # each rank calibrates on its own two batches (the oracle's statistics)
        qm, rb = O.measure_state(), {"running_mean": torch.zeros(8), "running_var": torch.zeros(8),
                                     "measure": O.measure_state()}
        for j in range(2):
            O.calibrate_measure(qm, synthetic.input_batch((3, 4, 6, 6), 500 + 10 * r + j))
            O.calibrate_rangebn(rb, synthetic.input_batch((4, 8, 6, 6), 700 + 10 * r + j))
        return qm, rb

    qm, rb = states(rank)
    with torch.no_grad():
        for k, v in qm.items():
            getattr(model[0].quantize_input, k).copy_(v)
        model[1].running_mean.copy_(rb["running_mean"])
        model[1].running_var.copy_(rb["running_var"])
        for k, v in rb["measure"].items():
            getattr(model[1].quantize_input, k).copy_(v)
    allreduce_calibration(model)
    both = [states(r) for r in range(world)]
    ok = True
    for k in ("running_min", "running_max", "running_mean", "running_var"):
        want = sum(s[0][k] for s in both) / world
        ok &= torch.allclose(getattr(model[0].quantize_input, k), want, rtol=1e-6, atol=0)
    for k in ("running_mean", "running_var"):
        ok &= torch.allclose(getattr(model[1], k), sum(s[1][k] for s in both) / world, rtol=1e-6, atol=0)
    # running-average momentum: the merged range is the one-process calibration over all batches
    seq = O.measure_state()
    for r in range(world):
        for j in range(2):
            O.calibrate_measure(seq, synthetic.input_batch((3, 4, 6, 6), 500 + 10 * r + j))
    ok &= torch.allclose(model[0].quantize_input.running_min, seq["running_min"], rtol=1e-6, atol=0)
    ok &= torch.allclose(model[0].quantize_input.running_max, seq["running_max"], rtol=1e-6, atol=0)
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_calibration_world2():
    """qnn.dist.allreduce_calibration averages every QuantMeasure / RangeBN running
    statistic over the ranks in one all-reduce."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_calib_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(q.get(timeout=10) for _ in range(2)) == [(0, True), (1, True)]


def test_async_gather_world1_keeps_every_step():
    """World size 1 (no process group): submit() still copies the engine's static logits
    into a send slot, so handles read after later forwards return their own step's logits."""
    w = torch.randn(16, 5, generator=torch.Generator().manual_seed(3))
    xs = [torch.randn(6, 16, generator=torch.Generator().manual_seed(200 + k)) for k in range(5)]
    runner = ShardedInference(_StaticEngine(6, w), 6)
    assert runner.world == 1
    handles = [runner.submit(x) for x in xs]
    outs = [h.result() for h in handles]
    assert all(torch.allclose(o, x @ w, rtol=0, atol=1e-5) for o, x in zip(outs, xs))
    assert all(o.data_ptr() != runner.model.logits.data_ptr() for o in outs)


def _calib_ragged_worker(rank, world, port, sizes, q):
    from oracle import qnn_oracle as O
    from qnn import synthetic
    from qnn.dist import allreduce_calibration
    from qnn.quantize import QuantMeasure
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    qmod = QuantMeasure(8)
    batches = [synthetic.input_batch((sum(sizes), 4, 6, 6), 900 + j) for j in range(2)]
    s = sum(sizes[:rank])
    st = O.measure_state()
    for b in batches:  # this rank's shard of each global calibration batch
        O.calibrate_measure(st, b[s:s + sizes[rank]])
    with torch.no_grad():
        for k, v in st.items():
            getattr(qmod, k).copy_(v)
    allreduce_calibration(qmod, samples=sizes[rank])
    one = O.measure_state()  # one process over the whole global batches
    for b in batches:
        O.calibrate_measure(one, b)
    ok = all(torch.allclose(getattr(qmod, k), one[k], rtol=2e-6, atol=0)
             for k in ("running_min", "running_max", "running_mean"))
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_calibration_ragged_shards_weighted():
    """Ragged shards (3 and 2 samples per batch): the sample-weighted merge of the extrema
    means and the mean equals a one-process calibration over the global batches."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_calib_ragged_worker, args=(r, 2, port, (3, 2), q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(q.get(timeout=10) for _ in range(2)) == [(0, True), (1, True)]


def _calib_weights_worker(rank, world, port, weights, q):
    from qnn.dist import allreduce_calibration
    from qnn.quantize import QuantMeasure
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    qmod = QuantMeasure(8)
    with torch.no_grad():
        qmod.running_min.fill_(float("-inf") if weights[rank] == 0 else -1.0 - rank)
        qmod.running_max.fill_(2.0 + rank)
    try:
        allreduce_calibration(qmod, samples=weights[rank])
        q.put((rank, "ok", float(qmod.running_min), float(qmod.running_max)))
    except ValueError:
        q.put((rank, "ValueError", None, None))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("weights,expect", [
    ((0, 4), ("ok", -2.0, 3.0)),            # a rank with no calibration samples takes part with weight 0
    ((-1, 4), ("ValueError", None, None)),  # an invalid weight raises on EVERY rank (no rank hangs)
    ((0, 0), ("ValueError", None, None)),
])
def test_allreduce_calibration_weights_collective(weights, expect):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_calib_weights_worker, args=(r, 2, port, weights, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert [r[1:] for r in res] == [expect, expect]


def _build_engine_fail_worker(rank, world, port, q):
    import qnn.engine as E
    from qnn.dist import build_engine

    class _Boom:  # stands in for qnn.Engine: rank 0's autotune fails (e.g. no tile configuration)
        def __init__(self, *a, **k):
            raise RuntimeError("no tile configuration")

    E.Engine = _Boom
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        build_engine(torch.nn.Identity(), 4)
        q.put((rank, "returned"))
    except RuntimeError as ex:
        q.put((rank, "raised", "no tile configuration" in str(ex) if rank == 0 else True))
    dist.barrier()
    dist.destroy_process_group()


def test_build_engine_rank0_failure_raises_on_every_rank():
    """rank 0's Engine construction failing must not leave the other ranks waiting in
    the tile-table broadcast -- every rank raises after the one collective."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_build_engine_fail_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(q.get(timeout=10) for _ in range(2)) == [(0, "raised", True), (1, "raised", True)]
