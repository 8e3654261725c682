"""The fragment-major operand layout of the MNIST tile path (hpnn_amd.ops.to_fragment_major:
the first-layer gradient's operands and the tile front's input), checked element by element
against its definition and round-tripped."""
import torch

from hpnn_amd import ops


def test_fragment_major_definition_and_inverse():
    Bt, M = 64, 48
    A = torch.arange(Bt * M, dtype=torch.int32).view(Bt, M)
    F = ops.to_fragment_major(A).view(Bt // 32, M // 16, 64, 8)  # [t][cb][g][r][j] as lanes
    for t in range(Bt // 32):
        for cb in range(M // 16):
            for lane in (0, 15, 17, 48, 63):
                g, r = lane // 16, lane % 16
                for j in range(8):
                    assert F[t, cb, lane, j] == A[32 * t + 8 * g + j, 16 * cb + r]
    assert torch.equal(ops.from_fragment_major(F, Bt, M), A)
