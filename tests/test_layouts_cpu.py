"""Operand layouts of the MNIST tile path (hpnn_amd.ops): fragment-major (the first-layer
gradient's, k = batch) and row-fragment-major (the tile front's, k = features), checked
element by element against their definitions and round-tripped."""
import torch

from hpnn_amd import ops


def test_row_fragment_major_definition_and_inverse():
    Bt, K = 64, 96
    A = torch.arange(Bt * K, dtype=torch.int32).view(Bt, K)
    R = ops.to_row_fragment_major(A)
    assert R.shape == (Bt // 16, K // 32, 64, 8)
    for u in range(Bt // 16):
        for s in range(K // 32):
            for lane in (0, 5, 16, 37, 63):
                h, r = lane // 16, lane % 16
                for j in range(8):
                    assert R[u, s, lane, j] == A[16 * u + r, 32 * s + 8 * h + j]
    assert torch.equal(ops.from_row_fragment_major(R, Bt, K), A)


def test_fragment_major_definition_and_inverse():
    Bt, M = 64, 48
    A = torch.arange(Bt * M, dtype=torch.int32).view(Bt, M)
    F = ops.to_fragment_major(A).view(Bt // 32, M // 16, 64, 8)  # [t][cb][g][r][j] as lanes
    assert F.shape == (Bt // 32, M // 16, 64, 8)
    for t in range(Bt // 32):
        for cb in range(M // 16):
            for lane in (0, 15, 17, 48, 63):
                g, r = lane // 16, lane % 16
                for j in range(8):
                    assert F[t, cb, lane, j] == A[32 * t + 8 * g + j, 16 * cb + r]
    assert torch.equal(ops.from_fragment_major(F, Bt, M), A)
