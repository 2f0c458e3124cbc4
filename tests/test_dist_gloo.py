"""Data-parallel harness (qnn/dist.py) on CPU with the gloo backend, world_size 2.

The GPU path is the same code with backend "nccl" (RCCL); only the collective's
transport differs.  Checks: contiguous ragged sharding, gather-to-root equals
the unsharded forward, non-root ranks get None, batch independence.
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
