"""Multi-rank paths with device tensors, at world size 2 on the one GPU of a box: both ranks
are freshly spawned processes on cuda:0 joined by the gloo backend (RCCL refuses two ranks on
one device; the 8-GPU RCCL path is the same code with backend "nccl").

* §8(f4) training under DistributedDataParallel (reference qdistiler_main.py:882-891): each
  rank runs the quantized model's training step (int8 forward, straight-through quantizers,
  8-bit stochastic gradient quantization) on its shard inside DDP; the averaged gradients must
  equal the mean of the ranks' plain (non-DDP) shard gradients (same stochastic draws).
* the data-parallel eval path (reference main.py:344-345, nn.DataParallel): each rank
  calibrates on its own shard, allreduce_calibration merges the statistics (sample-weighted),
  a qnn.Engine runs the rank's shard and ShardedInference gathers the logits on rank 0; they
  must equal, bitwise, one engine over the whole batch built from the same merged statistics.
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

FIXTURE = "model_resnet18_cifar"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(target, args, world=2, timeout=240):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=timeout)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, f"rank exit codes {codes}"


def _init(rank, world, port):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "quantized.pytorch_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from qnn import _lib
    _lib.load()
    return dist


# ---------------------------------------------------------------- DDP training step
GB_TRAIN = 8


def _train_batch(dev):
    from qnn import synthetic
    x = synthetic.input_batch((GB_TRAIN, 3, 32, 32), 77).to(dev)
    y = (torch.arange(GB_TRAIN, device=dev) * 3) % 10
    return x, y


def _shard_grads(model, x, y, seed):
    """One training step's gradients of `model` on (x, y), the stochastic draws from `seed`."""
    import torch.nn.functional as F
    torch.manual_seed(seed)
    model.zero_grad(set_to_none=True)
    F.cross_entropy(model(x), y).backward()


def _ddp_worker(rank, world, port, out):
    dist = _init(rank, world, port)
    from conftest import load_fixture
    from fixtures_util import build_model
    from qnn.dist import shard_bounds
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    dev = torch.device("cuda:0")
    x, y = _train_batch(dev)
    s, e = shard_bounds(GB_TRAIN, world, rank)
    # this rank's shard gradient without DDP, in this process (its own convolution algorithms)
    plain, _ = build_model(load_fixture(FIXTURE))
    plain = plain.to(dev).train()
    _shard_grads(plain, x[s:e], y[s:e], 100 + rank)
    model, _ = build_model(load_fixture(FIXTURE))
    model = model.to(dev).train()
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0], output_device=0)
    _shard_grads(ddp, x[s:e], y[s:e], 100 + rank)
    torch.save({"ddp": {n: p.grad.detach().cpu() for n, p in model.named_parameters()},
                "plain": {n: p.grad.detach().cpu() for n, p in plain.named_parameters()}}, f"{out}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_training_step_world2(gpu, tmp_path):
    """DDP's gradient on every rank is the world mean of the ranks' own shard gradients.

    Each rank computes its plain (non-DDP) shard gradient in its own process with the same
    stochastic draws, so the comparison does not depend on which convolution algorithms a
    process picked: across processes those may differ in the last bits, and the 8-bit
    stochastic gradient quantizer turns such a difference into a whole quantum (a first run
    comparing against gradients computed in the test process differed by one quantum, 2.4 %
    of max|grad|, on conv1.weight)."""
    out = str(tmp_path / "ddp_grads.pt")
    _spawn(_ddp_worker, (out,))
    got = [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]
    ddp, per = got[0]["ddp"], [g["plain"] for g in got]
    assert set(ddp) == set(per[0]) == set(got[1]["ddp"])
    worst = 0.0
    for n in ddp:
        assert torch.equal(ddp[n], got[1]["ddp"][n]), f"{n}: the ranks' averaged gradients differ"
        ref = (per[0][n] + per[1][n]) / 2  # DDP: every rank's gradient averaged over the world
        scale = ref.abs().max().item() + 1e-30
        err = (ddp[n] - ref).abs().max().item()
        worst = max(worst, err / scale)
        assert err <= 1e-6 * scale, f"{n}: max|d grad| {err:.3e} vs max|grad| {scale:.3e}"
        assert ref.abs().sum().item() > 0, n
    assert any(not torch.equal(per[0][n], per[1][n]) for n in ddp), "the two shards gave the same gradients"
    print(f"DDP world 2: {len(ddp)} parameter gradients, worst relative difference {worst:.2e}")


# ---------------------------------------------------------------- sharded eval engine
GB_EVAL = 7  # ragged: shards of 4 and 3 samples


def _calib_batches(rank, world):
    from qnn import synthetic
    from qnn.dist import shard_bounds
    s, e = shard_bounds(GB_EVAL, world, rank)
    return [synthetic.input_batch((GB_EVAL, 3, 32, 32), 500 + j)[s:e] for j in range(2)]


def _calibrate(model, batches, dev):
    from qnn.quantize import set_measure_mode
    set_measure_mode(model, True)
    model.train()
    with torch.no_grad():
        for b in batches:
            model(b.to(dev))
    set_measure_mode(model, False)
    model.eval()


def _eval_worker(rank, world, port, out):
    dist = _init(rank, world, port)
    from conftest import load_fixture
    from fixtures_util import build_model
    from qnn import synthetic
    from qnn.dist import ShardedInference, allreduce_calibration, build_engine, shard_bounds
    dev = torch.device("cuda:0")
    model, _ = build_model(load_fixture(FIXTURE))
    model = model.to(dev)
    batches = _calib_batches(rank, world)
    _calibrate(model, batches, dev)
    allreduce_calibration(model, samples=batches[0].shape[0])
    s, e = shard_bounds(GB_EVAL, world, rank)
    eng = build_engine(model, e - s)  # rank 0 autotunes, rank 1 runs its tiles
    torch.save(([k for k, _ in eng.tiles], getattr(eng, "tiles_fallback", [])), f"{out}.tiles{rank}")
    runner = ShardedInference(eng, GB_EVAL)
    x = synthetic.input_batch((GB_EVAL, 3, 32, 32), 600).to(dev)
    logits = runner(x[s:e])
    if rank == 0:
        torch.save({"logits": logits.detach().cpu(),
                    "state": {k: v.detach().cpu() for k, v in model.state_dict().items()}}, out)
    else:
        assert logits is None
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_engine_world2_device(gpu, tmp_path):
    from conftest import load_fixture
    from fixtures_util import build_model
    from qnn import synthetic
    from qnn.engine import Engine
    from qnn.quantize import QuantMeasure, RangeBN
    out = str(tmp_path / "eval.pt")
    _spawn(_eval_worker, (out,))
    got = torch.load(out, weights_only=True)
    (t0, _), (t1, fb1) = [torch.load(f"{out}.tiles{r}", weights_only=True) for r in range(2)]
    # rank 1 runs rank 0's configuration wherever it is built for rank 1's (ragged) shard
    assert all(a == b for n, (a, b) in enumerate(zip(t0, t1)) if n not in fb1), (t0, t1, fb1)
    # single process: each shard's calibration on its own, merged with the sample weights
    states = []
    for r in range(2):
        model, _ = build_model(load_fixture(FIXTURE))
        model = model.to(gpu)
        _calibrate(model, _calib_batches(r, 2), gpu)
        states.append(model)
    w = [b[0].shape[0] for b in (_calib_batches(0, 2), _calib_batches(1, 2))]
    merged = states[0]
    with torch.no_grad():
        for (n, m0), m1 in zip(merged.named_modules(), [m for _, m in states[1].named_modules()]):
            names = (("running_min", "running_max", "running_mean", "running_var") if isinstance(m0, QuantMeasure)
                     else ("running_mean", "running_var") if isinstance(m0, RangeBN) else ())
            for k in names:
                a, b = getattr(m0, k), getattr(m1, k)
                v = (a.double() * w[0] + b.double() * w[1]) / (w[0] + w[1])
                # the per-shard statistics recomputed in this process agree with the ranks' to the
                # device reduction's last bits (its fp64 partial sums are added in arrival order),
                # so the merge is checked to 1e-5 here and the engine below runs the ranks' own
                # merged state, bitwise
                ranks = got["state"][n + "." + k if n else k]
                rel = ((ranks.double() - v.cpu()).abs() / v.cpu().abs().clamp_min(1e-30)).max().item()
                assert torch.allclose(ranks.double(), v.cpu(), rtol=1e-5, atol=1e-12), f"merged {n}.{k}: rel {rel:.3g}"
                a.copy_(ranks.to(a.device))
    eng = Engine(merged, batch=GB_EVAL)
    ref = eng(synthetic.input_batch((GB_EVAL, 3, 32, 32), 600).to(gpu)).clone().cpu()
    assert got["logits"].shape == ref.shape
    ndiff = int((got["logits"] != ref).sum())
    assert ndiff == 0, f"{ndiff} gathered logits differ from the single-process engine"


# ---------------------------------------------------------------- C5 at world 2
# BASELINE.json configs[4] (C5): resnet_quantized depth=50, global batch 2048 sharded over 8 GPUs
# (per-rank batch 256) with one RCCL gather of the logits.  One box has one GPU, so the same code
# runs at world 2 (gloo, two ranks on cuda:0) at the C5 per-rank batch: each rank calibrates on
# its shard, allreduce_calibration merges, build_engine plans the rank's b256 engine with rank 0's
# autotuned tiles, ShardedInference gathers -- once with even shards (2 x 256) and once ragged
# (256 + 255).  Reference: nn.DataParallel at main.py:342-343.
C5_FIXTURE = "model_resnet50_imagenet"
C5_CASES = (512, 511)  # global batches: even and ragged shards at the per-rank batch 256
C5_CALIB = 32  # two shards of 16: RangeBN's chunked statistics need B*H*W % 16 == 0 at 7x7


def _c5_calib_batches(rank, world):
    from qnn import synthetic
    from qnn.dist import shard_bounds
    s, e = shard_bounds(C5_CALIB, world, rank)
    return [synthetic.input_batch((C5_CALIB, 3, 224, 224), 700 + j)[s:e] for j in range(2)]


def _c5_input(gb):
    from qnn import synthetic
    return synthetic.input_batch((gb, 3, 224, 224), 800 + gb)


def _c5_worker(rank, world, port, out):
    dist = _init(rank, world, port)
    from conftest import load_fixture
    from fixtures_util import build_model
    from qnn.dist import ShardedInference, allreduce_calibration, build_engine, shard_bounds
    dev = torch.device("cuda:0")
    model, _ = build_model(load_fixture(C5_FIXTURE))
    model = model.to(dev)
    batches = _c5_calib_batches(rank, world)
    _calibrate(model, batches, dev)
    allreduce_calibration(model, samples=batches[0].shape[0])
    res = {}
    for gb in C5_CASES:
        s, e = shard_bounds(gb, world, rank)
        print(f"[c5 rank {rank}] global batch {gb}: building the b{e - s} engine", flush=True)
        eng = build_engine(model, e - s)  # rank 0 autotunes, the other rank runs its tiles
        runner = ShardedInference(eng, gb)
        logits = runner(_c5_input(gb)[s:e].to(dev))
        res[gb] = {"tiles": [k for k, _ in eng.tiles], "shard": (s, e),
                   "logits": None if logits is None else logits.detach().cpu()}
        if rank != 0:
            assert logits is None
        del runner, eng
        torch.cuda.empty_cache()
    res["state"] = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    torch.save(res, f"{out}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_sharded_engine_world2_c5_resnet50(gpu, tmp_path):
    """C5's data path at world 2 and the C5 per-rank batch: the gathered logits of the sharded
    engines equal, bitwise, one engine over the whole global batch built from the same merged
    calibration (even and ragged shards)."""
    from conftest import load_fixture
    from fixtures_util import build_model
    from qnn.dist import shard_bounds
    from qnn.engine import Engine
    out = str(tmp_path / "c5.pt")
    _spawn(_c5_worker, (out,), timeout=800)
    got = [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]
    assert [got[r][512]["shard"] for r in range(2)] == [(0, 256), (256, 512)]
    assert [got[r][511]["shard"] for r in range(2)] == [(0, 256), (256, 511)]
    # every rank holds the same merged calibration after allreduce_calibration (its sample-weighted
    # merge is checked bitwise against a single-process reconstruction by
    # test_sharded_engine_world2_device above); the reference engine below is built from it
    s0, s1 = got[0]["state"], got[1]["state"]
    assert set(s0) == set(s1)
    for k in s0:
        assert torch.equal(s0[k], s1[k]), f"ranks disagree on {k} after the merge"
    merged, _ = build_model(load_fixture(C5_FIXTURE))
    merged.load_state_dict(s0, strict=True)
    merged = merged.to(gpu).eval()
    for gb in C5_CASES:
        # rank 1 ran rank 0's tile configuration wherever it is built for its shard
        t0, t1 = got[0][gb]["tiles"], got[1][gb]["tiles"]
        assert len(t0) == len(t1)
        eng = Engine(merged, batch=gb, autotune=False)  # the cost model's tiles: bitwise all the same
        ref = eng(_c5_input(gb).to(gpu)).clone().cpu()
        del eng
        torch.cuda.empty_cache()
        logits = got[0][gb]["logits"]
        assert logits.shape == ref.shape == (gb, 1000)
        ndiff = int((logits != ref).sum())
        assert ndiff == 0, f"global batch {gb}: {ndiff} gathered logits differ from the single-process engine"
        print(f"C5 world 2, global batch {gb} (shards {shard_bounds(gb, 2, 0)}, {shard_bounds(gb, 2, 1)}): "
              f"gathered logits bitwise the single-process engine")
