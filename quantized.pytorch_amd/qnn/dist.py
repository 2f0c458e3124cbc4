"""Data-parallel inference over the GPUs of one node: one process per GPU.

The reference's multi-GPU eval is single-process `nn.DataParallel`
(main.py:344-345): every forward scatters the batch, re-broadcasts all
parameters and buffers to every replica, runs replicas in threads and gathers
the outputs to device 0.  Here:
  * one process per GPU (torchrun env: RANK / LOCAL_RANK / WORLD_SIZE);
  * weights are loaded/packed once per rank (no per-forward broadcast);
  * each rank owns a contiguous slice of the global batch (inputs generated or
    loaded on that rank's device);
  * the only data-path collective is ONE gather of the logits to rank 0 over
    RCCL (`torch.distributed` backend "nccl" is RCCL on ROCm; xGMI on MI355X),
    issued asynchronously (`submit`): the logits are copied into one of two send
    slots and the gather overlaps the next step's forward;
  * calibration (main.py:154-205, measure mode) runs on every rank's own batches
    and `allreduce_calibration` merges the running statistics with ONE bucketed
    all-reduce, weighted by each rank's samples per batch (the reference's
    DataParallel keeps replica 0's statistics only, main.py:345).  The merged
    running_min / running_max / running_mean are exactly the statistics of all
    ranks' samples (means of per-sample or per-element values); QuantMeasure's std
    and RangeBN's inverse-range scale are nonlinear in the batch, so their merge is
    the sample-weighted mean of the per-rank values, an approximation.
The shard/gather logic is backend-agnostic and is tested with `gloo` on CPU.
"""
import os

import torch
import torch.distributed as dist


def env_rank():
    """(rank, local_rank, world_size) from the torchrun environment (defaults 0,0,1)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def init(backend=None):
    """Initialise the process group when WORLD_SIZE > 1; returns (rank, local_rank, world)."""
    rank, local_rank, world = env_rank()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    return rank, local_rank, world


def shard_bounds(global_batch, world, rank):
    """Contiguous [start, end) of rank's samples; sizes differ by at most one."""
    base, rem = divmod(global_batch, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def allreduce_calibration(model, group=None, samples=1):
    """Merge every calibrated statistic of `model` over the ranks of `group`: the
    running_min / running_max / running_mean / running_var of each QuantMeasure and the
    running_mean / running_var of each RangeBN, weighted by `samples` (this rank's samples
    per calibration batch: its shard size), flattened into one fp32 bucket and all-reduced
    once (RCCL on GPU tensors, gloo on CPU).  Call after every rank ran the same number
    of measure-mode batches.  Exact for the extrema means and the means; the std and the
    RangeBN scale merge as weighted means (module docstring).  No-op for world size 1.
    A rank with samples == 0 takes part with weight 0 (its buffers are ignored); invalid
    weights (negative, or every rank 0) raise ValueError on EVERY rank, after the one
    collective, so no rank is left waiting in it."""
    from .quantize import QuantMeasure, RangeBN
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    bufs = []
    for m in model.modules():
        if isinstance(m, QuantMeasure):
            bufs += [m.running_min, m.running_max, m.running_mean, m.running_var]
        elif isinstance(m, RangeBN):
            bufs += [m.running_mean, m.running_var]
    if not bufs:
        return
    w = float(samples) if samples > 0 else 0.0
    dev = bufs[0].device
    vals = torch.cat([b.detach().reshape(-1).to(torch.float64) for b in bufs])
    vals = vals * w if w > 0 else torch.zeros_like(vals)  # weight 0: never 0 * inf = nan
    flat = torch.cat([vals, torch.tensor([w, 1.0 if samples < 0 else 0.0], dtype=torch.float64, device=dev)])
    if dist.get_backend(group) == "gloo":
        flat = flat.cpu()  # gloo is the host transport (device buffers are staged through it)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    if flat[-1].item() > 0 or flat[-2].item() <= 0:
        raise ValueError("allreduce_calibration: samples must be >= 0 on every rank and > 0 on at least one")
    flat = flat[:-2] / flat[-2]
    off = 0
    with torch.no_grad():
        for b in bufs:
            n = b.numel()
            b.copy_(flat[off:off + n].view_as(b))
            off += n


def build_engine(model, batch, group=None, **kw):
    """A qnn.Engine for this rank whose tile configurations are rank 0's: rank 0 autotunes
    (times every configuration on its device) and broadcasts its choice, the other ranks plan
    with it instead of timing their own -- so every rank of a data-parallel job runs the same
    kernels (no per-rank timing skew in a max-over-ranks measurement; bitwise the same either
    way, every configuration computes identical outputs).  World size 1: a plain Engine."""
    from .engine import Engine
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return Engine(model, batch, **kw)
    rank = dist.get_rank(group)
    eng, err = None, None
    if rank == 0:
        try:
            eng = Engine(model, batch, **kw)
        except Exception as ex:  # noqa: BLE001 -- re-raised below, after the other ranks learn of it
            err = ex
    # n = -1 tells the other ranks that rank 0 failed, so no rank is left waiting in the
    # second broadcast; every rank then raises
    n = torch.tensor([len(eng.tiles) if eng is not None else -1 if err is not None else 0], dtype=torch.int64)
    dev_comm = dist.get_backend(group) == "nccl"
    if dev_comm:
        n = n.cuda()
    dist.broadcast(n, 0, group=group)
    if int(n.item()) < 0:
        if err is not None:
            raise err
        raise RuntimeError("build_engine: rank 0 failed to build its Engine (see rank 0's error)")
    t = torch.tensor([k for k, _ in eng.tiles] if eng is not None else [0] * int(n.item()), dtype=torch.int64)
    if dev_comm:
        t = t.cuda()
    dist.broadcast(t, 0, group=group)
    if eng is None:
        eng = Engine(model, batch, tiles=[int(v) for v in t.cpu().tolist()], **kw)
    return eng


class _Pending:
    """An in-flight gather (ShardedInference.submit): result() waits and returns the
    [global_batch, ...] logits on root, None elsewhere."""

    def __init__(self, work, fn):
        self._work, self._fn, self._out, self._done = work, fn, None, False

    def result(self):
        if not self._done:
            if self._work is not None:
                self._work.wait()
            self._out, self._done = self._fn(), True
        return self._out


class ShardedInference:
    """Run `model` on this rank's shard and gather the logits on `root`.

    `__call__(x_local)` returns the full [global_batch, ...] output on root and
    None elsewhere.  `submit(x_local)` issues the same gather asynchronously and
    returns a handle (`.result()`): the logits are first copied into one of two send
    slots, so the caller may start the next forward (which overwrites an engine's
    static logits) while the collective runs.  Ragged shards are padded to the
    largest shard for the collective and trimmed on root.
    """

    def __init__(self, model, global_batch, root=0, group=None):
        self.model = model
        self.global_batch = global_batch
        self.root = root
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.bounds = [shard_bounds(global_batch, self.world, r) for r in range(self.world)]
        self.max_shard = max(e - s for s, e in self.bounds)
        self._slots = {}  # shape -> [(send, recv list, pending handle)] x 2
        self._k = 0
        planned = getattr(model, "N", None)  # a qnn.Engine runs exactly the batch it was built for
        if planned is not None:
            s, e = self.bounds[self.rank]
            if e - s != planned:
                raise ValueError(f"rank {self.rank}: shard of {e - s} samples but the engine is planned for "
                                 f"{planned}; build each rank's Engine with its shard size")

    def local_slice(self):
        return self.bounds[self.rank]

    def submit_output(self, y_local):
        """Start gathering this rank's output `y_local`; returns a _Pending."""
        n_local = y_local.shape[0]
        s, e = self.bounds[self.rank]
        assert n_local == e - s, f"rank {self.rank}: expected a shard of {e - s}, got {n_local}"
        shape = (self.max_shard,) + tuple(y_local.shape[1:])
        slots = self._slots.get(shape)
        if slots is None:
            slots = self._slots[shape] = [None, None]
        k = self._k % 2
        self._k += 1
        # gloo is the host transport: device outputs are staged through host slots (RCCL moves
        # device buffers directly over xGMI)
        host = self.world > 1 and y_local.is_cuda and dist.get_backend(self.group) == "gloo"
        if slots[k] is None:
            send = torch.zeros(shape, dtype=y_local.dtype) if host else y_local.new_zeros(shape)
            recv = [torch.empty_like(send) for _ in range(self.world)] if self.rank == self.root else None
            slots[k] = [send, recv, None]
        send, recv, prev = slots[k]
        if prev is not None:
            prev.result()  # the gather that used this slot two submits ago has finished
        send[:n_local].copy_(y_local)  # ordered before the collective on the current stream
        if self.world == 1:  # no collective: the slot holds the copy until its handle is read
            slots[k][2] = pend = _Pending(None, lambda: send[:n_local].clone())
            return pend
        work = dist.gather(send, recv, dst=self.root, group=self.group, async_op=True)
        if self.rank == self.root:
            dev = y_local.device
            fn = lambda: torch.cat([b[: e_ - s_] for b, (s_, e_) in zip(recv, self.bounds)]).to(dev)
        else:
            fn = lambda: None
        slots[k][2] = pend = _Pending(work, fn)
        return pend

    def gather(self, y_local):
        return self.submit_output(y_local).result()

    def submit(self, x_local):
        with torch.no_grad():
            return self.submit_output(self.model(x_local))

    def __call__(self, x_local):
        with torch.no_grad():
            return self.gather(self.model(x_local))


class AbiComm:
    """The library's own RCCL communicator (include/qnn.h qnn_comm_*): the logits gather
    through the C ABI, for callers that bind the library without torch.distributed's
    collectives.  Rank 0 makes the id; it reaches the other ranks over the
    existing process group (any backend) when world > 1."""

    def __init__(self, rank=0, world=1):
        import ctypes
        from . import _lib
        self.rank, self.world = rank, world
        uid = (ctypes.c_ubyte * _lib.COMM_ID_BYTES)()
        if rank == 0:
            _lib.call("qnn_comm_unique_id", ctypes.byref(uid), ctypes.sizeof(uid))
        if world > 1:
            t = torch.tensor(list(uid), dtype=torch.uint8)
            if dist.get_backend() == "nccl":
                t = t.cuda()
            dist.broadcast(t, 0)
            uid = (ctypes.c_ubyte * _lib.COMM_ID_BYTES)(*t.cpu().tolist())
        _lib.call("qnn_comm_init", rank, world, ctypes.byref(uid))

    def gather(self, send, recv=None, root=0):
        """recv[r * send.numel():...] = rank r's send on the root, on the current stream."""
        from . import _lib
        assert send.is_contiguous() and send.dtype == torch.float32
        if self.rank == root:
            assert recv is not None and recv.numel() >= send.numel() * self.world and recv.is_contiguous()
        _lib.call("qnn_gather_f32", _lib.ptr(send), _lib.ptr(recv) if recv is not None else None, send.numel(),
                  root, _lib.stream_of(send))
        return recv

    def close(self):
        from . import _lib
        _lib.call("qnn_comm_destroy")
