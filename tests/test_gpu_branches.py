"""The engine's concurrent residual branches (qnn.Engine branches=True): each block's downsample
contraction runs on a second stream, forked after the block input and joined before the block's
last conv (the graph holds the two paths as parallel branches).  The logits must be bitwise those
of the serial launch order, eager and replayed, for the basic-block and bottleneck ResNets."""
import pytest
import torch

import bench
from qnn import synthetic
from qnn.engine import Engine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("depth,batch", [(18, 8), (50, 4)])
def test_branches_bitwise_vs_serial(gpu, depth, batch):
    model = bench.build(gpu, depth)
    x = synthetic.input_batch((batch, 3, 224, 224), 77).to(gpu)
    ser = Engine(model, batch, autotune=False, branches=False)
    par = Engine(model, batch, autotune=False, branches=True)
    assert par.forks and par.branches and not ser.branches
    assert len(par.forks) == (3 if depth == 18 else 4)
    with torch.no_grad():
        ref = ser(x).clone()
        for _ in range(3):  # replays: the forks and joins are graph edges
            assert torch.equal(par(x), ref)
        par.graph = None  # eager launch order through the side stream
        assert torch.equal(par(x), ref)
