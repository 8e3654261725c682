"""Numerics of the gfx950 kernels against plain PyTorch FP32 references."""
import os

import pytest
import torch

from hpnn_amd import ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _rand(*shape, scale=1.0, dev="cuda"):
    return ((torch.rand(*shape, device=dev) * 2 - 1) * scale)


@pytest.mark.parametrize("M,N,K", [(128, 32, 32), (256, 64, 64), (384, 128, 800), (128, 96, 96), (256, 256, 4096),
                                   (128, 32, 64), (256, 160, 224)])
@pytest.mark.parametrize("epi", [ops.EPI_NONE, ops.EPI_ACT, ops.EPI_DACT])
def test_gemm_nt(gpu, M, N, K, epi):
    torch.manual_seed(M + N + K + epi)
    A = _rand(M, K).bfloat16()
    # asymmetric B so a transposed store cannot pass
    B = (_rand(N, K) + torch.arange(N, device="cuda")[:, None] * 0.01).bfloat16()
    aux = _rand(M, N).bfloat16() if epi == ops.EPI_DACT else None
    for f32 in (False, True):
        C = ops.gemm_nt(A, B, epi, aux=aux, out_f32=f32)
        R = ops.ref_gemm_nt(A, B, epi, aux)
        tol = 2e-2 if not f32 else 2e-3
        err = (C.float() - R).abs().max().item()
        scale = R.abs().max().item() + 1e-6
        assert err <= tol * max(1.0, scale), (f32, err, scale)


@pytest.mark.parametrize("M,N,K", [(16384, 128, 800), (16416, 64, 800), (32768, 128, 512), (16384, 128, 1024),
                                   (65536, 128, 800)])
@pytest.mark.parametrize("epi", [ops.EPI_NONE, ops.EPI_ACT])
def test_gemm_nt_weight_stationary(gpu, M, N, K, epi):
    """large-batch shapes that take the weight-stationary kernel (kernels_ws.hip); M=16416
    leaves a ragged tile count over the persistent grid; X has a padded row stride."""
    torch.manual_seed(M + N + K)
    Xs = _rand(M, K + 64).bfloat16()
    A = Xs[:, :K]
    B = (_rand(N, K) + torch.arange(N, device="cuda")[:, None] * 0.01).bfloat16()
    for f32 in (False, True):
        C = ops.gemm_nt(A, B, epi, out_f32=f32)
        R = ops.ref_gemm_nt(A, B, epi, None)
        tol = 2e-2 if not f32 else 2e-3
        err = (C.float() - R).abs().max().item()
        scale = R.abs().max().item() + 1e-6
        assert err <= tol * max(1.0, scale), (f32, err, scale)


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 512), (8192, 2048, 640), (4352, 4096, 576), (16384, 256, 2048),
                                   (4096, 1024, 4096)])
@pytest.mark.parametrize("epi", [ops.EPI_NONE, ops.EPI_ACT, ops.EPI_DACT])
def test_gemm_nt_big_tile(gpu, M, N, K, epi):
    """shapes with >= 256 tiles of 256x256 take the 8-phase kernel (K % 128 == 0) or the
    1-phase large-tile kernel (K = 576); 64 tiles with a long K (16384 x 256 x 2048,
    4096 x 1024 x 4096) take the 128x128 kernel (the split-K form with HPNN_NT_SPLITK=1);
    padded row strides on every operand"""
    torch.manual_seed(M + N + K + epi)
    A = _rand(M, K + 64).bfloat16()[:, :K]
    B = (_rand(N, K + 32) + torch.arange(N, device="cuda")[:, None] * 0.001).bfloat16()[:, :K]
    aux = _rand(M, N + 32).bfloat16()[:, :N] if epi == ops.EPI_DACT else None
    for f32 in (False, True):
        out = torch.empty(M, N + 64, dtype=torch.float32 if f32 else torch.bfloat16, device="cuda")[:, :N]
        C = ops.gemm_nt(A, B, epi, aux=aux, out_f32=f32, out=out)
        R = ops.ref_gemm_nt(A, B, epi, aux)
        tol = 2e-2 if not f32 else 2e-3
        err = (C.float() - R).abs().max().item()
        scale = R.abs().max().item() + 1e-6
        assert err <= tol * max(1.0, scale), (f32, err, scale)


@pytest.mark.parametrize("M,N,K", [(1024, 4096, 4096), (1024, 512, 64), (384, 256, 128), (128, 128, 192)])
@pytest.mark.parametrize("epi", [ops.EPI_NONE, ops.EPI_ACT, ops.EPI_DACT])
def test_gemm_nt_pipelined_128(gpu, M, N, K, epi):
    """grids under two 128 x 128 tiles per CU take the software-pipelined kernel
    (kernels_mfma.hip gemm_nt_pp_kernel): against the FP32 reference, and BITWISE against the
    two-barrier kernel it replaces (same MFMA order per accumulator); K from one 64-wide step
    (no steady state) to 64 steps; padded row strides"""
    from hpnn_amd._lib import native
    torch.manual_seed(M + N + K + epi)
    A = _rand(M, K + 64).bfloat16()[:, :K]
    B = (_rand(N, K + 32) + torch.arange(N, device="cuda")[:, None] * 0.001).bfloat16()[:, :K]
    aux = _rand(M, N + 32).bfloat16()[:, :N] if epi == ops.EPI_DACT else None
    for f32 in (False, True):
        outs = []
        for pp in (1, 0):
            native().gemm_nt_set_pp(pp)
            try:
                out = torch.empty(M, N + 64, dtype=torch.float32 if f32 else torch.bfloat16, device="cuda")[:, :N]
                outs.append(ops.gemm_nt(A, B, epi, aux=aux, out_f32=f32, out=out))
            finally:
                native().gemm_nt_set_pp(1)
        R = ops.ref_gemm_nt(A, B, epi, aux)
        tol = 2e-2 if not f32 else 2e-3
        err = (outs[0].float() - R).abs().max().item()
        scale = R.abs().max().item() + 1e-6
        assert err <= tol * max(1.0, scale), (f32, err, scale)
        assert torch.equal(outs[0], outs[1]), f32


@pytest.mark.parametrize("M,N,K", [(1024, 4096, 4096), (1024, 512, 64), (384, 256, 128), (2048, 1024, 512)])
@pytest.mark.parametrize("epi", [ops.EPI_NONE, ops.EPI_ACT, ops.EPI_DACT])
def test_gemm_nn_matches_nt_on_transpose(gpu, M, N, K, epi):
    """C = epi(A . W) with W row-major [K][N] (kernels_mfma.hip gemm_nt_pp_kernel<..., BT>: W staged
    as a T32 image, read with the transposing LDS read) == the NT GEMM on the explicit W^T,
    BITWISE (the delta GEMM of the sharded data-parallel step reads W without its transposed
    copy); padded row strides"""
    from hpnn_amd._lib import native
    torch.manual_seed(M + N + K + epi)
    A = _rand(M, K + 64).bfloat16()[:, :K]
    W = (_rand(K, N + 32) + torch.arange(N + 32, device="cuda")[None, :] * 0.001).bfloat16()[:, :N]
    Wt = W.t().contiguous()
    aux = _rand(M, N + 32).bfloat16()[:, :N] if epi == ops.EPI_DACT else None
    s = torch.cuda.current_stream().cuda_stream
    for f32 in (False, True):
        dt = torch.float32 if f32 else torch.bfloat16
        C = torch.empty(M, N + 64, dtype=dt, device="cuda")[:, :N]
        native().gemm_nn_bf16(A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0), C.data_ptr(), C.stride(0),
                              aux.data_ptr() if aux is not None else 0, aux.stride(0) if aux is not None else 0,
                              M, N, K, epi, int(f32), s)
        R = ops.gemm_nt(A, Wt, epi, aux=aux, out_f32=f32)
        assert torch.equal(C, R), f32


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 512, 256), (768, 512, 384), (256, 1024, 1152),
                                   (2304, 256, 640)])
@pytest.mark.parametrize("epi", [ops.EPI_NONE, ops.EPI_ACT, ops.EPI_DACT])
def test_gemm_nt8(gpu, M, N, K, epi):
    """the 8-phase 256x256 kernel (kernels_8ph.hip) called directly at small grids: one
    iteration (K = 128, no restaging), odd iteration counts, a ragged XCD split (9 tiles),
    padded row strides on every operand"""
    from hpnn_amd._lib import native
    _check_nt8(native, M, N, K, epi)


def _check_nt8(native, M, N, K, epi):
    torch.manual_seed(M + 3 * N + K + epi)
    A = _rand(M, K + 64).bfloat16()[:, :K]
    B = (_rand(N, K + 32) + torch.arange(N, device="cuda")[:, None] * 0.001).bfloat16()[:, :K]
    aux = _rand(M, N + 32).bfloat16()[:, :N] if epi == ops.EPI_DACT else None
    for f32 in (False, True):
        C = torch.full((M, N + 64), float("nan"), dtype=torch.float32 if f32 else torch.bfloat16, device="cuda")[:, :N]
        native().gemm_nt8_bf16(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0),
                               aux.data_ptr() if aux is not None else 0, aux.stride(0) if aux is not None else 0,
                               M, N, K, epi, int(f32), torch.cuda.current_stream().cuda_stream)
        R = ops.ref_gemm_nt(A, B, epi, aux)
        tol = 2e-2 if not f32 else 2e-3
        err = (C.float() - R).abs().max().item()
        scale = R.abs().max().item() + 1e-6
        assert err <= tol * max(1.0, scale), (f32, err, scale)


@pytest.mark.parametrize("M,N,K,S", [(512, 256, 1024, 2), (256, 512, 768, 3), (1024, 256, 4096, 8), (256, 256, 256, 2)])
@pytest.mark.parametrize("epi", [ops.EPI_NONE, ops.EPI_ACT, ops.EPI_DACT])
def test_gemm_nt8_splitk(gpu, M, N, K, S, epi):
    """split-K form (FP32 slabs in the library workspace + one epilogue pass)"""
    from hpnn_amd._lib import native
    torch.manual_seed(M + N + K + S + epi)
    A = _rand(M, K + 64).bfloat16()[:, :K]
    B = (_rand(N, K + 32) + torch.arange(N, device="cuda")[:, None] * 0.001).bfloat16()[:, :K]
    aux = _rand(M, N + 32).bfloat16()[:, :N] if epi == ops.EPI_DACT else None
    for f32 in (False, True):
        C = torch.full((M, N + 64), float("nan"), dtype=torch.float32 if f32 else torch.bfloat16, device="cuda")[:, :N]
        native().gemm_nt8_splitk_bf16(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0),
                                      aux.data_ptr() if aux is not None else 0, aux.stride(0) if aux is not None else 0,
                                      M, N, K, epi, int(f32), S, torch.cuda.current_stream().cuda_stream)
        R = ops.ref_gemm_nt(A, B, epi, aux)
        tol = 2e-2 if not f32 else 2e-3
        err = (C.float() - R).abs().max().item()
        scale = R.abs().max().item() + 1e-6
        assert err <= tol * max(1.0, scale), (f32, err, scale)


def test_gemm_nt8_rejects_bad_shapes(gpu):
    from hpnn_amd._lib import native
    A = torch.zeros(256, 192, dtype=torch.bfloat16, device="cuda")
    C = torch.zeros(256, 256, dtype=torch.bfloat16, device="cuda")
    with pytest.raises(RuntimeError):
        native().gemm_nt8_bf16(A.data_ptr(), 192, A.data_ptr(), 192, C.data_ptr(), 256, 0, 0, 256, 256, 192,
                               ops.EPI_NONE, 0, torch.cuda.current_stream().cuda_stream)


def test_gemm_nt_identity(gpu):
    """A = I checks the C layout with an asymmetric B (cdna guide section 3)."""
    M, N, K = 128, 64, 128
    A = torch.eye(M, K, device="cuda").bfloat16()
    B = torch.arange(N * K, device="cuda", dtype=torch.float32).remainder(97).view(N, K).bfloat16()
    C = ops.gemm_nt(A, B, out_f32=True)
    assert torch.equal(C, B.float().t()[:M])


def test_gemm_nt_strided(gpu):
    M, N, K = 256, 64, 96
    A_big = _rand(M, 160).bfloat16()
    A = A_big[:, :K]
    B = _rand(N, K).bfloat16()
    C = ops.gemm_nt(A, B, out_f32=True)
    R = ops.ref_gemm_nt(A, B)
    assert (C - R).abs().max().item() < 2e-3 * R.abs().max().item() + 1e-4


@pytest.mark.parametrize("Bt,N,M,S", [(64, 32, 32, 1), (256, 64, 64, 2), (512, 128, 800, 4), (1024, 32, 128, 8),
                                      (256, 96, 160, 1), (2048, 256, 256, 4)])
def test_gemm_tn(gpu, Bt, N, M, S):
    torch.manual_seed(Bt + N + M)
    D = (_rand(Bt, N) + torch.arange(N, device="cuda")[None, :] * 0.01).bfloat16()
    H = _rand(Bt, M).bfloat16()
    slab = ops.gemm_tn(D, H, splits=S)
    G = slab.sum(0)
    R = ops.ref_gemm_tn(D, H)
    assert (G - R).abs().max().item() <= 1e-3 * R.abs().max().item() + 1e-4
    # each slab is its own batch slice
    c = Bt // S
    R0 = ops.ref_gemm_tn(D[:c], H[:c])
    assert (slab[0] - R0).abs().max().item() <= 1e-3 * R0.abs().max().item() + 1e-4


@pytest.mark.parametrize("Bt,N,M,S", [(1024, 4096, 4096, 1), (2048, 2048, 4096, 2), (640, 4096, 2048, 3),
                                      (128, 4096, 4096, 1), (512, 2048, 2048, 4), (384, 4096, 4096, 1)])
def test_gemm_tn_big_tile(gpu, Bt, N, M, S):
    """>= 256 tiles of 256x256 take the large-tile kernels: the 8-phase one (kernels_8ph.hip)
    when every split holds an even number of 64-row units (one iteration: Bt = 128 and
    the 4-split case; several: Bt = 1024, 2048), else the 4-stage 8-wave kernel (640 / 3,
    384 = 6 units is even -> 8-phase with 3 iterations); padded strides, uneven splits"""
    torch.manual_seed(Bt + N + M)
    D = (_rand(Bt, N + 32) + torch.arange(N + 32, device="cuda")[None, :] * 0.001).bfloat16()[:, :N]
    H = _rand(Bt, M + 64).bfloat16()[:, :M]
    slab = ops.gemm_tn(D, H, splits=S)
    R = ops.ref_gemm_tn(D, H)
    assert (slab.sum(0) - R).abs().max().item() <= 1e-3 * R.abs().max().item() + 1e-4
    a, b = ops.split_rows(Bt, S)[S - 1]
    R1 = ops.ref_gemm_tn(D[a:b], H[a:b])
    assert (slab[S - 1] - R1).abs().max().item() <= 1e-3 * R1.abs().max().item() + 1e-4


@pytest.mark.parametrize("Bt,S", [(640, 3), (65536 // 8, 12), (1024, 16)])
def test_gemm_tn_uneven_splits(gpu, Bt, S):
    """split s covers the 64-row units [s*U/S, (s+1)*U/S): slabs match the row ranges"""
    torch.manual_seed(S)
    N, M = 128, 800
    D = _rand(Bt, N).bfloat16()
    H = _rand(Bt, M).bfloat16()
    slab = ops.gemm_tn(D, H, splits=S)
    rows = ops.split_rows(Bt, S)
    assert rows[0][0] == 0 and rows[-1][1] == Bt and len({b - a for a, b in rows}) <= 2
    for s_ in (0, S // 2, S - 1):
        a, b = rows[s_]
        R = ops.ref_gemm_tn(D[a:b], H[a:b])
        assert (slab[s_] - R).abs().max().item() <= 1e-3 * R.abs().max().item() + 1e-4
    R = ops.ref_gemm_tn(D, H)
    assert (slab.sum(0) - R).abs().max().item() <= 1e-3 * R.abs().max().item() + 1e-4


@pytest.mark.parametrize("S", [1, 8, 96, 37])
def test_reduce_slabs_many(gpu, S):
    torch.manual_seed(S)
    slab = torch.randn(S, 128, 800, device="cuda")
    out = torch.empty(128, 800, device="cuda")
    ops.reduce_slabs(slab, out)
    assert torch.allclose(out, slab.double().sum(0).float(), atol=1e-4, rtol=1e-5)
    ops.reduce_slabs(slab, out)
    out2 = out.clone()
    ops.reduce_slabs(slab, out)
    assert torch.equal(out, out2)  # deterministic


def _sgd_multi_case(momentum, seed=11):
    torch.manual_seed(seed)
    layers, refs = [], []
    # (32, 64, 3) and (64, 96, 1): layers with fewer than 8 slabs next to a 96-slab layer,
    # so some waves of the sub-tile kernel hold no slab at all
    for i, (N, K, S) in enumerate([(128, 800, 96), (64, 128, 16), (32, 64, 9), (32, 64, 3), (64, 96, 1)]):
        W = torch.randn(N, K, device="cuda")
        V = torch.randn(N, K, device="cuda") * 0.1 if momentum else None
        G = torch.randn(S, N, K, device="cuda")
        Wb = torch.empty(N, K, dtype=torch.bfloat16, device="cuda")
        Wt = torch.empty(K, N, dtype=torch.bfloat16, device="cuda")
        Wf = torch.empty(N * K, dtype=torch.bfloat16, device="cuda") if i == 0 else None
        refs.append((W.double().clone(), None if V is None else V.double().clone(), G.double().sum(0)))
        layers.append((W, V, G, Wb, Wt, Wf))
    return layers, refs


@pytest.mark.parametrize("momentum", [False, True])
def test_sgd_update_multi_wide(gpu, momentum):
    """many slabs (>= 8): the 8-row sub-tile kernel; same step as the FP64 reference,
    bitwise repeatable.  Runs in a child process whose environment drops HPNN_UPD_NARROW
    (read once per process)."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("HPNN_UPD_NARROW",)}
    code = ("import sys, importlib.util as u; sys.path.insert(0, %r); "
            "s = u.spec_from_file_location('tk', %r); t = u.module_from_spec(s); s.loader.exec_module(t); "
            "t._sgd_multi_check(%r)" % (ROOT, os.path.abspath(__file__), momentum))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr


def _sgd_multi_check(momentum):
    layers, refs = _sgd_multi_case(momentum)
    lr, alpha, scale = 0.05, 0.2, 1.0 / 512
    ops.sgd_update_multi(layers, lr, alpha, scale, momentum)
    torch.cuda.synchronize()
    again, _ = _sgd_multi_case(momentum)
    ops.sgd_update_multi(again, lr, alpha, scale, momentum)
    torch.cuda.synchronize()
    assert torch.equal(again[0][0], layers[0][0])  # deterministic
    assert torch.equal(layers[0][5], ops.frag_major(layers[0][0].bfloat16()))
    for (W, V, G, Wb, Wt, _), (W0, V0, g) in zip(layers, refs):
        if momentum:
            v = V0 + lr * g * scale
            w = W0 + v
            assert torch.allclose(V.double(), v * alpha, atol=1e-5)
        else:
            w = W0 + lr * g * scale
        assert torch.allclose(W.double(), w, atol=1e-5)
        assert torch.equal(Wb, W.bfloat16()) and torch.equal(Wt, W.bfloat16().t())


def test_gemm_tn_integer_exact(gpu):
    """small integers are exact in bf16/fp32: any index permutation shows up."""
    Bt, N, M = 128, 32, 64
    D = torch.randint(-3, 4, (Bt, N), device="cuda").float().bfloat16()
    H = torch.randint(-3, 4, (Bt, M), device="cuda").float().bfloat16()
    G = ops.gemm_tn(D, H, splits=2).sum(0)
    assert torch.equal(G, ops.ref_gemm_tn(D, H))


@pytest.mark.parametrize("net_type", [ops.TYPE_SNN, ops.TYPE_ANN, ops.TYPE_LNN])
@pytest.mark.parametrize("n_out,ldz,B", [(10, 32, 256), (230, 256, 256), (64, 64, 256), (100, 128, 256),
                                        (150, 160, 256), (256, 256, 256), (300, 320, 256), (230, 256, 20000),
                                        (4096, 4096, 512), (1001, 1024, 300)])
def test_output_delta(gpu, net_type, n_out, ldz, B):
    n_valid = B - 56
    torch.manual_seed(n_out + net_type)
    Z = _rand(B, ldz, scale=3.0)
    labels = torch.randint(0, n_out, (B,), device="cuda", dtype=torch.int32)
    hi, lo = (1.0, 0.0) if net_type == ops.TYPE_SNN else (1.0, -1.0)
    T = torch.full((B, n_out), lo, device="cuda")
    T[torch.arange(B), labels.long()] = hi
    D = torch.empty(B, ldz, dtype=torch.bfloat16, device="cuda")
    O = torch.empty(B, ldz, device="cuda")
    stats = torch.zeros(64, 16, device="cuda")  # HPNN_STAT_SLOTS x HPNN_STAT_STRIDE
    ops.output_delta(Z, n_out, net_type, D, labels=labels, t_hi=hi, t_lo=lo, n_valid=n_valid, O=O,
                     loss_acc=stats[0, 0:1], correct=stats[0, 1:2])
    loss = stats[:, 0].sum()
    corr = stats[:, 1].contiguous().view(torch.int32).sum()
    o, d, l = ops.ref_output(Z, n_out, net_type, T)
    assert (O[:, :n_out] - o).abs().max().item() < 1e-5
    assert (D[:n_valid, :n_out].float() - d[:n_valid]).abs().max().item() < 1e-2 * max(1, d.abs().max().item())
    assert D[n_valid:].float().abs().max().item() == 0.0
    if ldz > n_out:
        assert D[:, n_out:].float().abs().max().item() == 0.0
    assert abs(loss.item() - l[:n_valid].sum().item()) < 1e-3 * max(1.0, abs(l[:n_valid].sum().item()))
    hits = (o[:n_valid].argmax(1) == labels[:n_valid].long()).sum().item()
    assert corr.item() == hits
    # dense targets give the same delta
    D2 = torch.empty_like(D)
    ops.output_delta(Z, n_out, net_type, D2, T=T, n_valid=n_valid)
    assert torch.equal(D, D2)


@pytest.mark.parametrize("momentum", [False, True])
def test_sgd_update(gpu, momentum):
    N, K, S = 64, 96, 3
    W = _rand(N, K)
    V = _rand(N, K, scale=0.1) if momentum else None
    G = _rand(S, N, K)
    Wb = torch.empty(N, K, dtype=torch.bfloat16, device="cuda")
    Wt = torch.empty(K, N, dtype=torch.bfloat16, device="cuda")
    W0, V0 = W.clone(), (V.clone() if momentum else None)
    lr, alpha, scale = 0.05, 0.2, 1.0 / 7
    ops.sgd_update(W, V, G, Wb, Wt, lr, alpha, scale, momentum)
    g = G.sum(0) * scale
    if momentum:
        v = V0 + lr * g
        w = W0 + v
        v = v * alpha
        assert (V - v).abs().max().item() < 1e-6
    else:
        w = W0 + lr * g
    assert (W - w).abs().max().item() < 1e-6
    assert torch.equal(Wb, W.bfloat16())
    assert torch.equal(Wt, W.bfloat16().t())


def test_pack_bf16(gpu):
    X = torch.rand(100, 784, dtype=torch.float64, device="cuda")
    out = torch.full((128, 800), 7.0, dtype=torch.bfloat16, device="cuda")
    ops.pack_bf16(X, out)
    assert torch.equal(out[:100, :784], X.float().bfloat16())
    assert out[100:].abs().max().item() == 0 and out[:, 784:].abs().max().item() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("S,groups", [(256, 16), (100, 7), (5, 5)])
def test_gemm_tn_with_tail_reduce(gpu, S, groups):
    """gemm_tn + reduce_groups in one launch (reduction on appended workgroups) == the two
    separate kernels, bit for bit"""
    torch.manual_seed(S + groups)
    Bt, N, M = 65536, 128, 800
    D = _rand(Bt, N).bfloat16()
    H = _rand(Bt, M).bfloat16()
    sl = torch.randn(S, 10240, device="cuda")
    a_slab = torch.empty(48, N, M, device="cuda")
    b_slab = torch.empty_like(a_slab)
    a_red = torch.full((groups, 10240), float("nan"), device="cuda")
    b_red = torch.full_like(a_red, float("nan"))
    ops.gemm_tn(D, H, splits=48, out=a_slab)
    ops.reduce_groups(sl, groups, a_red)
    ops.gemm_tn_reduce(D, H, 48, b_slab, sl, groups, b_red)
    torch.cuda.synchronize()
    assert torch.equal(a_slab, b_slab)
    assert torch.equal(a_red, b_red)
