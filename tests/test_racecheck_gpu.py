"""Race detection on the GPU (hpnn_amd/utils/racecheck.py): repeated training runs from
the same state must give bit-identical FP32 weights and momentum on every path (fused
X->delta1 kernel, fused middle kernel, generic per-layer kernels), with batches that
exercise partial tiles.  A missing barrier or an LDS ring hazard shows up here as a
mismatch."""
import pytest
import torch

from hpnn_amd.models import MLP
from hpnn_amd.utils import racecheck


@pytest.mark.gpu
@pytest.mark.parametrize("sizes,fused,batch", [
    ([784, 128, 64, 10], "x", 8192),
    ([784, 128, 64, 10], "mid", 4096 + 384),
    ([300, 96, 40, 7], None, 3000),
    ([851, 230, 230], None, 2048),
])
def test_training_step_is_bitwise_deterministic(gpu, sizes, fused, batch):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11)
    Xr = [torch.rand(batch, sizes[0], device=dev, generator=g) for _ in range(2)]
    Ls = [torch.randint(0, sizes[-1], (batch,), device=dev, generator=g, dtype=torch.int32) for _ in range(2)]

    def mk():
        return MLP(sizes, "SNN", batch=batch, device=dev, momentum=True, seed=3,
                   fused=fused if fused else False)

    prepared = {}

    def bt(m, i):
        key = (id(m), i % 2)
        if key not in prepared:
            prepared[key] = m.prepare_input(Xr[i % 2])
        return prepared[key], Ls[i % 2]

    bad = racecheck.check(mk, bt, steps=4, repeats=3)
    assert all(not b for b in bad), bad
