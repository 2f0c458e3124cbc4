"""The C-ABI RCCL gather (include/qnn.h qnn_comm_*) on one GPU: a
world-1 communicator, the gather of a logits block to the root bitwise, argument checks.
(The multi-rank path is the driver's 8-GPU run; the shard/gather logic around it is the
gloo-tested qnn.dist.)"""
import pytest
import torch

from qnn import _lib
from qnn.dist import AbiComm

pytestmark = pytest.mark.gpu


def test_abi_gather_world1(gpu):
    comm = AbiComm(0, 1)
    try:
        x = torch.randn(37, 1000, device=gpu)
        y = torch.full_like(x, -1.0)
        comm.gather(x, y)
        torch.cuda.synchronize()
        assert torch.equal(x, y)
        # empty send: a no-op success
        comm.gather(x[:0].contiguous(), y)
        with pytest.raises(_lib.QnnError):
            _lib.call("qnn_gather_f32", _lib.ptr(x), _lib.ptr(y), x.numel(), 1, _lib.stream_of(x))  # root >= world
        with pytest.raises(_lib.QnnError):
            _lib.call("qnn_comm_init", 0, 1, None)  # null id
    finally:
        comm.close()
    with pytest.raises(_lib.QnnError):  # no communicator after destroy
        _lib.call("qnn_gather_f32", _lib.ptr(x), _lib.ptr(y), x.numel(), 0, _lib.stream_of(x))
