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
    RCCL (`torch.distributed` backend "nccl" is RCCL on ROCm; xGMI on MI355X).
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


class ShardedInference:
    """Run `model` on this rank's shard and gather the logits on `root`.

    `__call__(x_local)` returns the full [global_batch, ...] output on root and
    None elsewhere.  Ragged shards are padded to the largest shard for the
    collective and trimmed on root.
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
        self._gather_bufs = None
        planned = getattr(model, "N", None)  # a qnn.Engine runs exactly the batch it was built for
        if planned is not None:
            s, e = self.bounds[self.rank]
            if e - s != planned:
                raise ValueError(f"rank {self.rank}: shard of {e - s} samples but the engine is planned for "
                                 f"{planned}; build each rank's Engine with its shard size")

    def local_slice(self):
        return self.bounds[self.rank]

    def gather(self, y_local):
        if self.world == 1:
            return y_local
        n_local = y_local.shape[0]
        s, e = self.bounds[self.rank]
        assert n_local == e - s, f"rank {self.rank}: expected a shard of {e - s}, got {n_local}"
        if n_local != self.max_shard:
            pad = y_local.new_zeros((self.max_shard - n_local,) + tuple(y_local.shape[1:]))
            y_send = torch.cat([y_local, pad])
        else:
            y_send = y_local.contiguous()
        if self.rank == self.root:
            if self._gather_bufs is None or self._gather_bufs[0].shape != y_send.shape:
                self._gather_bufs = [torch.empty_like(y_send) for _ in range(self.world)]
            dist.gather(y_send, self._gather_bufs, dst=self.root, group=self.group)
            parts = [b[: e - s] for b, (s, e) in zip(self._gather_bufs, self.bounds)]
            return torch.cat(parts)
        dist.gather(y_send, None, dst=self.root, group=self.group)
        return None

    def __call__(self, x_local):
        with torch.no_grad():
            return self.gather(self.model(x_local))
