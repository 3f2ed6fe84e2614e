"""HIP kernel numerics vs plain-PyTorch fp32 references (run on an MI355X via gpurun).

Asymmetric operands (cdna_hip_programming.md §3: a symmetric/identity operand hides a
transposed fragment map) and shapes that are not tile multiples."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _lib():
    from nnmpi_amd import native
    return native.lib()


def _s():
    return torch.cuda.current_stream().cuda_stream


def _rand(*shape, dtype=torch.float32, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV, dtype)


def test_library_is_gfx950():
    assert _lib().arch().startswith("gfx950")


@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(64, 64, 64), (264, 136, 200), (128, 512, 512), (40, 24, 8)])
def test_gemm_layouts(la, lb, M, N, K):
    lib = _lib()
    A = _rand(M, K, seed=1).to(torch.bfloat16)
    B = _rand(K, N, seed=2).to(torch.bfloat16)
    # storage: KMAJ A = [M][K]; XMAJ A = [K][M]; KMAJ B = [N][K]; XMAJ B = [K][N]
    As = A.contiguous() if la == 0 else A.t().contiguous()
    Bs = B.t().contiguous() if lb == 0 else B.contiguous()
    C = torch.zeros(M, N, device=DEV)
    lib.gemm_bf16(As.data_ptr(), As.stride(0), la, Bs.data_ptr(), Bs.stride(0), lb, M, N, K,
                  C.data_ptr(), N, _s())
    ref = A.float() @ B.float()
    torch.testing.assert_close(C, ref, rtol=1e-4, atol=1e-3)


def test_gemm_identity_asymmetric():
    lib = _lib()
    M = N = K = 64
    A = torch.eye(64, device=DEV, dtype=torch.bfloat16)
    B = torch.arange(64 * 64, device=DEV, dtype=torch.float32).reshape(64, 64).remainder(97).to(torch.bfloat16)
    Bs = B.t().contiguous()
    C = torch.zeros(M, N, device=DEV)
    lib.gemm_bf16(A.data_ptr(), 64, 0, Bs.data_ptr(), 64, 0, M, N, K, C.data_ptr(), N, _s())
    torch.testing.assert_close(C, B.float())


def test_cu_mask_stream_runs_kernels_bitwise_equal():
    """cu_mask_stream (the CU-partitioned concurrency experiment, scripts/r4_cu_split_ab.py; an
    experiments-build entry point): a GEMM on a stream restricted to half the CUs gives the same
    bits as on the whole chip."""
    lib = _lib()
    if not lib.experiments_built():
        with pytest.raises(RuntimeError, match="experiments build only"):
            lib.cu_mask_stream([1])
        pytest.skip("the production library carries no experiment entry point")
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    mask = [0] * ((n_cu + 31) // 32)
    for c in range(0, n_cu, 2):
        mask[c // 32] |= 1 << (c % 32)
    st = lib.cu_mask_stream(mask)
    try:
        M, N, K = 1024, 768, 512
        A = _rand(M, K, seed=11).to(torch.bfloat16)
        Bs = _rand(N, K, seed=12).to(torch.bfloat16)
        C0 = torch.zeros(M, N, device=DEV)
        C1 = torch.zeros(M, N, device=DEV)
        lib.gemm_bf16(A.data_ptr(), K, 0, Bs.data_ptr(), K, 0, M, N, K, C0.data_ptr(), N, _s())
        torch.cuda.synchronize()
        lib.gemm_bf16(A.data_ptr(), K, 0, Bs.data_ptr(), K, 0, M, N, K, C1.data_ptr(), N, st)
        torch.cuda.ExternalStream(st).synchronize()
        assert torch.equal(C0, C1)
        torch.testing.assert_close(C0, A.float() @ Bs.float().t(), rtol=1e-4, atol=1e-3)
    finally:
        lib.stream_destroy(st)


@pytest.mark.parametrize("act", ["relu", "tanh", "none"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K", [(8192, 512, 512), (1000, 264, 136), (4097, 1024, 784)])
def test_linear_fwd(act, dtype, M, N, K):
    from nnmpi_amd.ops.hip_ops import HipOps
    from nnmpi_amd.ops.torch_ops import TorchOps
    x = _rand(M, K, seed=3).to(dtype)
    W = _rand(N, K, seed=4, scale=0.05).to(dtype)
    b = _rand(N, seed=5)
    out = torch.empty(M, N, device=DEV, dtype=dtype)
    ref = torch.empty(M, N, device=DEV, dtype=dtype)
    HipOps().linear_act(x, W, b, act, out)
    TorchOps(DEV).linear_act(x, W, b, act, ref)
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(out.float(), ref.float(), **tol)


@pytest.mark.parametrize("act", ["relu", "tanh"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K", [(8192, 512, 512), (1000, 264, 136)])
def test_linear_dgrad(act, dtype, M, N, K):
    from nnmpi_amd.ops.hip_ops import HipOps
    from nnmpi_amd.ops.torch_ops import TorchOps
    dz = _rand(M, K, seed=6).to(dtype)
    W = _rand(K, N, seed=7, scale=0.05).to(dtype)     # layer weight [out=K][in=N]
    a_prev = torch.relu(_rand(M, N, seed=8)).to(dtype) if act == "relu" else torch.tanh(_rand(M, N, seed=8)).to(dtype)
    out = torch.empty(M, N, device=DEV, dtype=dtype)
    ref = torch.empty(M, N, device=DEV, dtype=dtype)
    HipOps().linear_dgrad(dz, W, a_prev, act, out)
    TorchOps(DEV).linear_dgrad(dz, W, a_prev, act, ref)
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(out.float(), ref.float(), **tol)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,out_f,in_f", [(8192, 512, 512), (8193, 512, 512), (100, 264, 136),
                                             (4096, 1024, 784)])
def test_linear_wgrad(dtype, rows, out_f, in_f):
    from nnmpi_amd.ops.hip_ops import HipOps
    ops = HipOps()
    dz = _rand(rows, out_f, seed=9).to(dtype)
    x = _rand(rows, in_f, seed=10).to(dtype)
    gW = torch.full((out_f, in_f), 7.0, device=DEV)
    gb = torch.full((out_f,), 7.0, device=DEV)
    ws = torch.zeros(ops.wgrad_workspace_bytes(rows, out_f, in_f, dtype) // 4 + 16, device=DEV)
    ops.linear_wgrad(dz, x, gW, gb, ws=ws)
    refW = dz.double().t() @ x.double()
    refb = dz.double().sum(0)
    scale = (rows ** 0.5)
    torch.testing.assert_close(gW.double(), refW, rtol=1e-3, atol=1e-3 * scale)
    torch.testing.assert_close(gb.double(), refb, rtol=1e-3, atol=1e-3 * scale)


@pytest.mark.parametrize("loss,out_f", [("mse", 1), ("mse", 3), ("xent", 10), ("xent", 100),
                                        ("mse", 37)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,in_f", [(8192, 512), (777, 1024), (64, 8192), (300, 100)])
def test_head(loss, out_f, dtype, rows, in_f):
    """Every head shape against the fp32 oracle: the skinny kernels (out <= 16, weights within
    64 KiB of LDS) and the general path (8192 -> 10 cross-entropy, 8192 -> 3 regression,
    100 classes, in % 8 != 0)."""
    from nnmpi_amd.ops.hip_ops import HipOps
    from nnmpi_amd.ops.torch_ops import TorchOps
    ops = HipOps()
    a = torch.relu(_rand(rows, in_f, seed=11)).to(dtype)
    W = _rand(out_f, in_f, seed=12, scale=0.05)
    b = _rand(out_f, seed=13)
    y = _rand(rows, out_f, seed=14) if loss == "mse" else None
    lab = (torch.arange(rows, device=DEV) * 7 % out_f) if loss == "xent" else None
    res = {}
    for name, o in (("hip", ops), ("ref", TorchOps(DEV))):
        gW = torch.zeros(out_f, in_f, device=DEV)
        gb = torch.zeros(out_f, device=DEV)
        dz = torch.zeros(rows, in_f, device=DEV, dtype=dtype)
        dl = torch.zeros(rows, out_f, device=DEV)
        lo = torch.zeros(4, device=DEV)
        ws = torch.zeros(ops.head_workspace_bytes(rows, in_f, out_f) // 4 + 16, device=DEV)
        o.head(a, W, b, y, lab, loss, 1.0 / rows, "relu", dz, gW, gb, dl, lo, 1.0 / rows, ws=ws)
        res[name] = (gW, gb, dz, lo[0], dl)
    tol = dict(rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(res["hip"][0], res["ref"][0], **tol)
    torch.testing.assert_close(res["hip"][1], res["ref"][1], **tol)
    if dtype == torch.bfloat16:
        _assert_dz_within_bf16_bound(res["hip"][2], res["ref"][2], res["ref"][4], W, a)
    else:
        torch.testing.assert_close(res["hip"][2], res["ref"][2], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(res["hip"][3], res["ref"][3], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("loss,out_f,rows,in_f,act", [("xent", 10, 8192, 1024, "relu"),
                                                      ("xent", 10, 777, 512, "tanh"),
                                                      ("mse", 3, 1000, 1024, "relu"),
                                                      ("xent", 16, 33, 1024, "relu")])
def test_multi_output_head_fused_matches_two_launch_path(loss, out_f, rows, in_f, act):
    """The fused multi-output head (logits, loss, dZ and the weight gradient in one kernel on the
    bf16 matrix cores, head_mo.hip) against the two-launch fp32-MFMA path (head_mfma_kernel +
    head_wgrad_mfma_kernel) on the same inputs: the fused kernel splits W and dl into bf16
    hi + lo terms for the logits and the weight gradient (~2^-16 relative), so loss, gW and gb
    agree to that; its dZ runs on bf16 dl and W like every hidden layer's dgrad and must stay
    inside the bf16 rounding bound of the fp32 reference."""
    from nnmpi_amd import native
    from nnmpi_amd.ops.hip_ops import HipOps
    from nnmpi_amd.ops.torch_ops import TorchOps
    lib = native.lib()
    assert lib.head_mo_fused_ok(1, rows, in_f, out_f, 1 if loss == "xent" else 0)
    ops = HipOps()
    a = torch.relu(_rand(rows, in_f, seed=41)).to(torch.bfloat16)
    if act == "tanh":
        a = torch.tanh(_rand(rows, in_f, seed=41)).to(torch.bfloat16)
    W = _rand(out_f, in_f, seed=42, scale=0.05)
    b = _rand(out_f, seed=43)
    y = _rand(rows, out_f, seed=44) if loss == "mse" else None
    lab = (torch.arange(rows, device=DEV) * 3 % out_f) if loss == "xent" else None
    res = {}
    try:
        for name, o, fused in (("fused", ops, 1), ("split", ops, 0), ("ref", TorchOps(DEV), 1)):
            if o is ops:
                assert lib.set_head_fused(fused)
            gW = torch.zeros(out_f, in_f, device=DEV)
            gb = torch.zeros(out_f, device=DEV)
            dz = torch.zeros(rows, in_f, device=DEV, dtype=torch.bfloat16)
            dl = torch.zeros(rows, out_f, device=DEV)
            lo = torch.zeros(4, device=DEV)
            ws = torch.full((ops.head_workspace_bytes(rows, in_f, out_f) // 4 + 16,), float("nan"),
                            device=DEV)
            o.head(a, W, b, y, lab, loss, 1.0 / rows, act, dz, gW, gb, dl, lo, 1.0 / rows, ws=ws)
            torch.cuda.synchronize()
            res[name] = (gW, gb, dz, lo[0].item(), dl)
    finally:
        lib.set_head_fused(-1)
    f, s, ref = res["fused"], res["split"], res["ref"]
    assert f[3] == pytest.approx(s[3], rel=2e-5)
    torch.testing.assert_close(f[0], s[0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(f[1], s[1], rtol=1e-4, atol=1e-5)
    _assert_dz_within_bf16_bound(f[2], ref[2], ref[4], W, a, act)


def _assert_dz_within_bf16_bound(dz, ref, dl, W, a, act="relu"):
    """dZ = (dl . W) * relu'(a) stored in bf16.  The matrix-core general head runs it as the bf16
    dgrad GEMM on bf16 copies of dl and W (fp32 accumulation), so every product carries at most
    two bf16 roundings (u = 2^-8 each) and the result one more, and the reference (itself stored
    in bf16) one: elementwise |dz - ref| <= 2u |ref| + (2u + u^2) sum_n |dl_n W_nf| (+ a denormal
    floor).  The exact fp32 kernels satisfy the tighter 2u |ref| part alone."""
    u = 2.0 ** -8
    # |act'(a)| scales each product: relu 0 / 1, tanh 1 - a^2 (of the bf16 activation)
    mask = (a.float() > 0).double() if act == "relu" else (1 - a.double() ** 2).abs()
    bound = (2 * u * ref.double().abs() + (2 * u + u * u) * (dl.double().abs() @ W.double().abs()) * mask
             + 1e-30) * 1.01
    err = (dz.double() - ref.double()).abs()
    worst = float((err / bound).max())
    assert worst <= 1.0, f"dZ outside the bf16 rounding bound: max err/bound {worst:.3f}"


@pytest.mark.parametrize("loss,out_f,rows,in_f", [("xent", 10, 1000, 8192), ("xent", 100, 777, 1024),
                                                 ("mse", 37, 300, 512), ("xent", 128, 64, 256)])
def test_general_head_matrix_core_path_vs_valu_path(loss, out_f, rows, in_f):
    """The matrix-core general head (bf16 activations) against the fp32 VALU general head on the
    same inputs: loss and dlogits to fp32 summation-order noise, the weight / bias gradient
    (fp32 MFMA on the fp32 dlogits) likewise, dZ to bf16 rounding (it runs the bf16 dgrad GEMM on
    bf16 dlogits and weights, like every hidden layer)."""
    from nnmpi_amd import native
    from nnmpi_amd.ops.hip_ops import HipOps
    lib = native.lib()
    assert lib.head_general_mfma_ok(1, in_f, out_f)
    ops = HipOps()
    a = torch.relu(_rand(rows, in_f, seed=31)).to(torch.bfloat16)
    W = _rand(out_f, in_f, seed=32, scale=0.05)
    b = _rand(out_f, seed=33)
    y = _rand(rows, out_f, seed=34) if loss == "mse" else None
    lab = (torch.arange(rows, device=DEV) * 5 % out_f) if loss == "xent" else None
    res = {}
    try:
        for valu in (0, 1):
            lib.set_head_general_valu(valu)
            gW = torch.zeros(out_f, in_f, device=DEV)
            gb = torch.zeros(out_f, device=DEV)
            dz = torch.zeros(rows, in_f, device=DEV, dtype=torch.bfloat16)
            dl = torch.zeros(rows, out_f, device=DEV)
            lo = torch.zeros(4, device=DEV)
            ws = torch.zeros(ops.head_workspace_bytes(rows, in_f, out_f) // 4 + 16, device=DEV)
            ops.head(a, W, b, y, lab, loss, 1.0 / rows, "relu", dz, gW, gb, dl, lo, 1.0 / rows, ws=ws)
            torch.cuda.synchronize()
            res[valu] = (gW, gb, dz, dl, lo[0].item())
    finally:
        lib.set_head_general_valu(0)
    m, v = res[0], res[1]
    assert m[4] == pytest.approx(v[4], rel=1e-5)
    torch.testing.assert_close(m[3], v[3], rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(m[0], v[0], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(m[1], v[1], rtol=1e-4, atol=1e-6)
    # the VALU path's dZ is the exact fp32 product rounded once; the MFMA path's is within the
    # bf16 dgrad bound of it
    _assert_dz_within_bf16_bound(m[2], v[2], v[3], W, a)


@pytest.mark.parametrize("first,nesterov,wd,damp", [(True, False, 0.0, 0.0), (False, False, 0.0, 0.0),
                                                    (False, True, 1e-2, 0.0), (False, False, 1e-2, 0.3)])
def test_sgd_matches_torch_optim(first, nesterov, wd, damp):
    from nnmpi_amd.engine.arena import Arena
    from nnmpi_amd.ops.hip_ops import HipOps
    ar = Arena([(64, 200), (1, 64)], DEV, shadow_dtype=torch.bfloat16)
    ar.master.copy_(_rand(ar.numel, seed=20))
    ar.grad.copy_(_rand(ar.numel, seed=21))
    ar.momentum.copy_(_rand(ar.numel, seed=22))
    p = torch.nn.Parameter(ar.master.clone())
    opt = torch.optim.SGD([p], lr=0.01, momentum=0.9, dampening=damp, weight_decay=wd, nesterov=nesterov)
    if not first:
        opt.state[p]["momentum_buffer"] = ar.momentum.clone()
    p.grad = ar.grad.clone() * 0.5
    opt.step()
    hp = torch.tensor([0.01, 0.9, damp, wd, 0.5, 0, 0, 0], device=DEV)
    HipOps().sgd(ar, hp, nesterov, first)
    torch.testing.assert_close(ar.master, p.detach(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(ar.momentum, opt.state[p]["momentum_buffer"], rtol=1e-6, atol=1e-6)
    assert torch.equal(ar.shadow, ar.master.to(torch.bfloat16))
    assert torch.count_nonzero(ar.grad) == 0


@pytest.mark.parametrize("M,N,K", [(1024, 512, 256), (520, 264, 200), (2048, 8192, 512)])
def test_wgrad_bf16_output_equals_cast_of_fp32(M, N, K):
    """The weight gradient stored as bf16 by its own epilogue == the fp32 gradient cast to bf16
    (the bf16 all-reduce payload), bit for bit, bias gradient included."""
    from nnmpi_amd.ops.hip_ops import HipOps
    ops = HipOps()
    assert ops.wgrad_can_write_bf16(K, M, N)
    dz = _rand(K, M, seed=40).to(torch.bfloat16)
    x = _rand(K, N, seed=41).to(torch.bfloat16)
    gW = torch.empty(M, N, device=DEV)
    gb = torch.empty(M, device=DEV)
    ops.linear_wgrad(dz, x, gW, gb)
    gW16 = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    gb16 = torch.full((M,), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.linear_wgrad(dz, x, None, None, out_bf16=(gW16, gb16))
    assert torch.equal(gW16, gW.to(torch.bfloat16))
    assert torch.equal(gb16, gb.to(torch.bfloat16))
    ref = dz.float().t() @ x.float()
    torch.testing.assert_close(gW16.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())


@pytest.mark.parametrize("first", [True, False])
def test_sgd_bf16_gradient_and_background_grid(first):
    """The bf16-gradient update (the overlapped schedule's bf16 payload) against torch.optim.SGD
    on the same bf16 values in fp32, and the fixed-grid launch against the default one."""
    from nnmpi_amd.engine.arena import Arena
    from nnmpi_amd.ops.hip_ops import HipOps
    ar = Arena([(64, 200), (1, 64)], DEV, shadow_dtype=torch.bfloat16)
    ar.master.copy_(_rand(ar.numel, seed=30))
    ar.grad.copy_(_rand(ar.numel, seed=31))
    ar.momentum.copy_(_rand(ar.numel, seed=32))
    g16 = _rand(ar.numel, seed=33).to(torch.bfloat16)
    m0, v0, g0 = ar.master.clone(), ar.momentum.clone(), ar.grad.clone()
    p = torch.nn.Parameter(m0.clone())
    opt = torch.optim.SGD([p], lr=0.01, momentum=0.9, weight_decay=1e-3)
    if not first:
        opt.state[p]["momentum_buffer"] = v0.clone()
    p.grad = g16.float() * 0.5
    opt.step()
    hp = torch.tensor([0.01, 0.9, 0.0, 1e-3, 0.5, 0, 0, 0], device=DEV)
    ops = HipOps()
    # two halves: offsets into the master/momentum/shadow AND the bf16 buffer
    h = (ar.numel // 2) // 4 * 4
    ops.sgd(ar, hp, False, first, offset=0, numel=h, grad_bf16=g16)
    ops.sgd(ar, hp, False, first, offset=h, numel=ar.numel - h, grad_bf16=g16)
    torch.testing.assert_close(ar.master, p.detach(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(ar.momentum, opt.state[p]["momentum_buffer"], rtol=1e-6, atol=1e-6)
    assert torch.equal(ar.shadow, ar.master.to(torch.bfloat16))
    assert torch.equal(ar.grad, g0), "the fp32 gradient arena must stay untouched"
    # the same update from the fp32 copy of those values is bitwise identical
    ar2 = Arena([(64, 200), (1, 64)], DEV, shadow_dtype=torch.bfloat16)
    ar2.master.copy_(m0)
    ar2.momentum.copy_(v0)
    ar2.grad.copy_(g16.float())
    ops.sgd(ar2, hp, False, first)
    assert torch.equal(ar2.master, ar.master) and torch.equal(ar2.momentum, ar.momentum)
    # fixed-grid ("background") launch == default launch, bitwise
    ar3 = Arena([(64, 200), (1, 64)], DEV, shadow_dtype=torch.bfloat16)
    ar3.master.copy_(m0)
    ar3.momentum.copy_(v0)
    ar3.grad.copy_(g16.float())
    _lib().sgd_momentum_bg(ar3.master.data_ptr(), ar3.grad.data_ptr(), ar3.momentum.data_ptr(),
                           ar3.shadow.data_ptr(), ar3.numel, hp.data_ptr(), 0, int(first), 1, 3,
                           torch.cuda.current_stream().cuda_stream)
    assert torch.equal(ar3.master, ar.master) and torch.equal(ar3.momentum, ar.momentum)
    assert torch.count_nonzero(ar3.grad) == 0


@pytest.mark.parametrize("tile", [256, 128])
@pytest.mark.parametrize("M,N,K", [(600, 520, 200), (4096, 1024, 512)])
def test_forced_tile_fwd_dgrad_wgrad(tile, M, N, K):
    """Every MLP GEMM orientation through a forced tile edge (256x256: the large-shape path),
    ragged M/N/K tails included."""
    from nnmpi_amd.ops.hip_ops import HipOps
    from nnmpi_amd.ops.torch_ops import TorchOps
    lib = _lib()
    ops, tops = HipOps(), TorchOps(DEV)
    x = _rand(M, K, seed=11).to(torch.bfloat16)
    W = _rand(N, K, seed=12, scale=0.05).to(torch.bfloat16)
    b = _rand(N, seed=13)
    dz = _rand(M, N, seed=14).to(torch.bfloat16)
    lib.set_gemm_tile(tile)
    try:
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.linear_act(x, W, b, "relu", out)
        dx = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
        ops.linear_dgrad(dz, W, x, "tanh", dx)
        gW, gb = torch.empty(N, K, device=DEV), torch.empty(N, device=DEV)
        ws = torch.empty(ops.wgrad_workspace_bytes(M, N, K, torch.bfloat16) // 4 + 64, device=DEV)
        ops.linear_wgrad(dz, x, gW, gb, ws=ws)
        torch.cuda.synchronize()
    finally:
        lib.set_gemm_tile(0)
    ref = torch.empty_like(out)
    tops.linear_act(x, W, b, "relu", ref)
    torch.testing.assert_close(out.float(), ref.float(), rtol=2e-2, atol=2e-2)
    rdx = torch.empty_like(dx)
    tops.linear_dgrad(dz, W, x, "tanh", rdx)
    torch.testing.assert_close(dx.float(), rdx.float(), rtol=2e-2, atol=2e-2)
    rgW, rgb = torch.empty_like(gW), torch.empty_like(gb)
    tops.linear_wgrad(dz, x, rgW, rgb)
    torch.testing.assert_close(gW, rgW, rtol=1e-3, atol=2e-2)
    torch.testing.assert_close(gb, rgb, rtol=1e-3, atol=2e-2)


def test_native_runtime_under_host_asan():
    """The C++ runtime (RCCL communicator, GradSync, GraphRunner, launchers) driven from a native
    binary built with host AddressSanitizer + UBSan (scripts/build_runtime_check.sh; device code
    is not instrumented).  Any ASan/UBSan report aborts the binary with a non-zero status."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "neural-networks-parallel-training-with-mpi_amd", "native_tests",
                       "runtime_check_asan")
    if not os.path.exists(exe):
        pytest.skip("runtime_check_asan not built (scripts/build_runtime_check.sh)")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=100, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ALL OK" in r.stdout


def _mix64(z):
    m = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & m
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & m
    return z ^ (z >> 31)


@pytest.mark.parametrize("n", [1, 7, 4096 * 4 + 3, 300_001])
def test_replica_hash_kernel_vs_host(n):
    """hash_u32 (the bench's replica check) == the host sum of splitmix64((i << 32) | word_i) mod
    2^64, for vector bodies and scalar tails; flipping any single bit changes it."""
    import numpy as np
    from nnmpi_amd import native
    lib = native.lib()
    g = torch.Generator().manual_seed(n)
    words = torch.randint(-2 ** 31, 2 ** 31 - 1, (n,), generator=g, dtype=torch.int64).to(torch.int32)
    x = words.cuda()
    out = torch.zeros(1025, dtype=torch.int64, device="cuda")
    lib.hash_u32(x.data_ptr(), n, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    got = int(out[1024].item()) & ((1 << 64) - 1)
    w = words.numpy().astype(np.int64) & 0xFFFFFFFF
    sample = range(n) if n < 5000 else None
    if sample is not None:
        ref = sum(_mix64((i << 32) | int(w[i])) for i in sample) & ((1 << 64) - 1)
        assert got == ref
    y = x.clone()
    k = n // 2
    y[k] = y[k] ^ (1 << (n % 31))
    lib.hash_u32(y.data_ptr(), n, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert (int(out[1024].item()) & ((1 << 64) - 1)) != got
