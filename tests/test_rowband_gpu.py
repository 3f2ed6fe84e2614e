"""Row-band step (csrc/kernels/rowband.hip): the forward, the MSE head and every activation
gradient of a narrow square regressor in one launch, the weight gradients in one grouped launch,
the combines (+ fused SGD) in one more.  Numerics against the plain-PyTorch fp32 oracle with the
same bf16 rounding contract (TorchOps), and against the grouped schedule it replaces."""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.rowband]


def _engine(widths, rows, dev, ops, *, seed=3, lr=0.0, momentum=0.0, fuse_sgd=True, rowband=None,
            monkeypatch=None, act="relu"):
    from nnmpi_amd.engine.arena import Arena
    from nnmpi_amd.engine.engine import MLPEngine
    from nnmpi_amd.models.mlp import MLPSpec, reference_init
    from nnmpi_amd.parallel.sync import NoSync
    spec = MLPSpec(tuple(widths), act, "mse")
    ar = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], dev, shadow_dtype=torch.bfloat16)
    ar.bind_model(reference_init(widths, act, seed=seed))
    if monkeypatch is not None and rowband is not None:
        monkeypatch.setenv("NNMPI_ROWBAND", "1" if rowband else "0")
    eng = MLPEngine(spec, ar, ops, NoSync(ar), device=dev, dtype=torch.bfloat16,
                    rows_capacity=rows, lr=lr, momentum=momentum, use_graph=False,
                    fuse_sgd=fuse_sgd)
    return spec, ar, eng


def _data(rows, widths, dev="cuda"):
    from nnmpi_amd.data import synth
    X, Y = synth.chunked_regression(0, rows, widths[0], out=1, device=dev)
    return X.to(torch.bfloat16), Y


_SHAPES = [([512, 512, 512, 512, 1], 1024, "relu"),
           ([512, 512, 512, 512, 1], 1000, "relu"),
           ([512, 512, 512, 1], 8191, "relu"),
           ([512, 512, 1], 37, "relu"),
           ([512, 512, 512, 512, 1], 777, "tanh"),
           ([512] * 5 + [1], 2048, "relu"),
           # other widths, input width != hidden width, 1-4 hidden layers
           ([256, 256, 256, 256, 1], 1000, "relu"),
           ([768, 768, 768, 1], 555, "tanh"),
           ([1024, 1024, 1024, 1], 1024, "relu"),
           ([256, 512, 512, 512, 1], 999, "relu"),
           ([1024, 512, 512, 1], 640, "tanh"),
           ([128, 384, 384, 1], 300, "tanh"),
           ([512, 256, 1], 64, "relu")]


@pytest.mark.parametrize("widths,rows,act", _SHAPES)
def test_rowband_gradients_vs_oracle(widths, rows, act, monkeypatch):
    """Every layer's weight and bias gradient, the activations, every dZ and the loss of ONE
    row-band step (no optimizer) vs the fp32 oracle: 1e-2 relative norm per tensor (a wrong
    scale on any layer, a missed row of a partial band or a transposed weight operand fails).
    The fragment-major weight images are built first (rowband_pack).  The band kernel itself
    (the column-split form off: NNMPI_RB_SPLIT=0)."""
    from nnmpi_amd import native
    lib = native.lib()
    assert lib.rowband_split_ok(1024, 512, 512, 3, 1)
    lib.set_rb_split(0)
    try:
        assert not lib.rowband_split_ok(rows, widths[1], widths[0], len(widths) - 2, 1)
        _oracle_check(widths, rows, act, monkeypatch)
    finally:
        lib.set_rb_split(-1)


# the column-split kernel's shapes: H = 512, in 256 / 512, 1-4 hidden layers, <= 4,096 rows
# (8 / 4 / 2 blocks per band at <= 1,024 / 2,048 / 4,096 rows)
_SPLIT_SHAPES = [([512, 512, 512, 512, 1], 1024, "relu", 0),
                 ([512, 512, 512, 512, 1], 1000, "relu", 0),
                 ([512, 512, 512, 512, 1], 2048, "relu", 0),
                 ([512, 512, 512, 512, 1], 4096, "relu", 0),
                 ([512, 512, 512, 512, 1], 3001, "relu", 0),
                 ([512, 512, 512, 512, 1], 3001, "tanh", 0),
                 ([512, 512, 512, 512, 1], 2047, "tanh", 0),
                 ([512, 512, 1], 37, "relu", 0),
                 ([512, 512, 512, 1], 64, "relu", 0),
                 ([512] * 5 + [1], 2047, "relu", 0),
                 ([256, 512, 512, 512, 1], 999, "relu", 0),
                 ([512, 512, 512, 512, 1], 777, "tanh", 0),
                 ([512, 512, 512, 512, 1], 1000, "relu", 4),
                 ([512, 512, 512, 512, 1], 1000, "relu", 2),
                 ([512, 512, 512, 512, 1], 2048, "relu", 2),
                 # the weight gradients' image path at other shapes (whole 8-band groups): one
                 # hidden layer, input width 256, 3 / 6 k-blocks per wave, four hidden layers
                 ([512, 512, 1], 256, "relu", 0),
                 ([256, 512, 512, 512, 1], 1024, "relu", 0),
                 ([512, 512, 512, 512, 1], 768, "tanh", 0),
                 ([512] * 5 + [1], 1536, "relu", 0)]


@pytest.mark.parametrize("widths,rows,act,groups", _SPLIT_SHAPES)
def test_rowband_split_gradients_vs_oracle(widths, rows, act, groups, monkeypatch):
    """The column-split row-band kernel (small batches: each band's columns over 2-8 blocks,
    activations exchanged per layer through write-through stores and per-band counters) vs the
    fp32 oracle, as the band kernel above; ``groups`` forces the blocks per band (0: automatic).
    The engine takes it by itself below the band kernel's row threshold; no wait timed out."""
    from nnmpi_amd import native
    lib = native.lib()
    monkeypatch.setenv("NNMPI_ROWBAND_MIN_ROWS", "6144")   # (the production threshold)
    if groups:
        lib.set_rb_split(groups)
    try:
        assert lib.rowband_split_ok(rows, widths[1], widths[0], len(widths) - 2, 1 if act == "relu" else 2)
        eng = _oracle_check(widths, rows, act, monkeypatch)
        assert eng.uses_rowband_split(rows) and eng.schedule_name() == "rowband"
        eng.check_device_errors()
    finally:
        lib.set_rb_split(-1)


@pytest.mark.parametrize("rows", [1024, 2047])
def test_rowband_small_wgrad_matches_the_slab_form(rows, monkeypatch):
    """The small-batch weight gradients (wgrad_small: un-split 64 x 64 tiles, SGD-momentum and
    the weight images in the epilogue, the head's combine in the same launch) against the split-K
    slabs + combine launch (NNMPI_RB_WGSMALL=0): three fused-update steps, parameters within
    1e-5 relative (different summation order), losses within 1e-4."""
    from nnmpi_amd import native
    from nnmpi_amd.ops.hip_ops import HipOps
    lib = native.lib()
    monkeypatch.setenv("NNMPI_ROWBAND_MIN_ROWS", "6144")
    widths = [512, 512, 512, 512, 1]
    X, Y = _data(rows, widths)
    res = []
    try:
        for small in (1, 0):
            assert lib.set_rb_wgsmall(small)
            _, ar, eng = _engine(widths, rows, "cuda", HipOps("cuda"), lr=1e-3, momentum=0.9,
                                 rowband=True, monkeypatch=monkeypatch)
            assert eng.uses_rowband_split(rows)
            eng.load_batch(X, Y)
            eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
            losses = []
            for _ in range(3):
                eng.step()
                losses.append(eng.loss())
            res.append((ar.master.double().cpu(), losses))
    finally:
        lib.set_rb_wgsmall(-1)
    (p1, l1), (p2, l2) = res
    assert float((p1 - p2).norm() / p2.norm()) < 1e-5
    for a, b in zip(l1, l2):
        assert a == pytest.approx(b, rel=1e-4)


@pytest.mark.parametrize("widths,rows", [([512, 512, 512, 512, 1], 1024), ([512, 512, 512, 512, 1], 2048),
                                         ([512, 512, 1], 256), ([256, 512, 512, 512, 1], 1000),
                                         ([512] * 5 + [1], 1536), ([512, 512, 512, 1], 3072),
                                         ([512, 512, 512, 512, 1], 4096)])
def test_rowband_small_wgrad_image_path_matches_the_lds_tiles(widths, rows, monkeypatch):
    """wgrad_small's image path (operands from the K-major fragments the split kernel writes,
    K split over the 8 waves, partial tiles summed in wave order; gemm_bf16.hip wgs_kimg_tile)
    against what runs without it (set_wgs_kimg(0)): the LDS-DMA tiles up to 2,048 rows, the
    split-K slabs + combine above: three fused-update steps, parameters within 1e-5 relative
    (different summation order), losses within 1e-4; no wait timed out."""
    from nnmpi_amd import native
    from nnmpi_amd.ops.hip_ops import HipOps
    lib = native.lib()
    monkeypatch.setenv("NNMPI_ROWBAND_MIN_ROWS", "6144")
    assert lib.wgrad_kimg_ok(rows)
    X, Y = _data(rows, widths)
    res = []
    try:
        for kimg in (1, 0):
            assert lib.set_wgs_kimg(kimg)
            _, ar, eng = _engine(widths, rows, "cuda", HipOps("cuda"), lr=1e-3, momentum=0.9,
                                 rowband=True, monkeypatch=monkeypatch)
            assert eng.uses_rowband_split(rows)
            eng.load_batch(X, Y)
            eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
            losses = []
            for _ in range(3):
                eng.step()
                losses.append(eng.loss())
            eng.check_device_errors()
            res.append((ar.master.double().cpu(), losses))
    finally:
        lib.set_wgs_kimg(-1)
    (p1, l1), (p2, l2) = res
    assert float((p1 - p2).norm() / p2.norm()) < 1e-5
    for a, b in zip(l1, l2):
        assert a == pytest.approx(b, rel=1e-4)


def _oracle_check(widths, rows, act, monkeypatch):
    from nnmpi_amd.ops.hip_ops import HipOps
    from nnmpi_amd.ops.torch_ops import TorchOps
    X, Y = _data(rows, widths)
    out = []
    for dev, ops in (("cuda", HipOps("cuda")), ("cpu", TorchOps("cpu"))):
        spec, ar, eng = _engine(widths, rows, dev, ops, rowband=True, monkeypatch=monkeypatch,
                                act=act)
        eng.load_batch(X.to(dev), Y.to(dev))
        eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
        L = spec.n_layers
        with torch.no_grad():
            if dev == "cuda":
                assert ops.rowband_version(rows, widths, act, "mse") == 2
                assert eng.rb_version == 2
                layers = [(ar.compute_weight(i), ar.bias(i), eng.acts[i][:rows], eng._dzl(i, rows),
                           ar.grad_weight(i), ar.grad_bias(i)) for i in range(L - 1)]
                kw = {}
                with torch.cuda.stream(eng.stream):
                    eng._rb_pack()
                    kw["packed"] = eng.rb_packed
                    ops.rowband_step(eng.X[:rows], layers, ar.weight(L - 1), ar.bias(L - 1),
                                     eng.Y[:rows], eng.inv_count, ar.grad_weight(L - 1),
                                     ar.grad_bias(L - 1), eng.ws_rb, eng.loss_scale, eng.loss_out,
                                     act, **kw)
                eng.synchronize()
            else:
                eng.forward_backward()
        rec = {("g", li, k): t.double().cpu().clone()
               for li in range(L) for k, t in enumerate((ar.grad_weight(li), ar.grad_bias(li)))}
        for i in range(L - 1):
            rec[("a", i)] = eng.acts[i][:rows].double().cpu().clone()
            rec[("dz", i)] = eng._dzl(i, rows).double().cpu().clone()
        rec["loss"] = float(eng.loss_out[0].item())
        out.append(rec)
        if dev == "cuda":
            geng = eng
    g, r = out
    assert g["loss"] == pytest.approx(r["loss"], rel=1e-3)
    for key in r:
        if key == "loss":
            continue
        a, b = g[key], r[key]
        rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
        assert rel < 1e-2, (key, rel)
    return geng


def test_rowband_engine_is_taken_and_trains_like_grouped(monkeypatch):
    """The engine takes the row-band schedule for the proxy shape; 5 SGD-momentum steps track the
    grouped schedule's trajectory (same math, different summation order: close, not bitwise)."""
    from nnmpi_amd.ops.hip_ops import HipOps
    widths, rows = [512, 512, 512, 512, 1], 2048
    X, Y = _data(rows, widths)
    res = []
    for rb in (True, False):
        spec, ar, eng = _engine(widths, rows, "cuda", HipOps("cuda"), lr=1e-3, momentum=0.9,
                                rowband=rb, monkeypatch=monkeypatch)
        assert eng.rowband == rb
        eng.load_batch(X, Y)
        eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
        losses = []
        for _ in range(5):
            eng.step()
            losses.append(eng.loss())
        res.append((losses, ar.master.double().cpu().clone()))
    (l1, p1), (l2, p2) = res
    for a, b in zip(l1, l2):
        assert a == pytest.approx(b, rel=2e-3)
    assert float((p1 - p2).norm() / p2.norm()) < 1e-4
    assert l1[-1] < l1[0]


@pytest.mark.parametrize("split", [False, True])
def test_rowband_fused_update_is_bitwise_equal_to_separate_pass(split, monkeypatch):
    """One rank: the combines apply SGD-momentum themselves; bitwise the same parameters as the
    row-band gradients followed by the standalone optimizer pass (same slab sums, same pinned
    update arithmetic).  ``split``: the small-batch path (column-split kernel + the un-split
    weight gradients with the update in their epilogue, wgrad_small)."""
    from nnmpi_amd.ops.hip_ops import HipOps
    widths, rows = [512, 512, 512, 512, 1], 1500
    if split:
        monkeypatch.setenv("NNMPI_ROWBAND_MIN_ROWS", "6144")
    X, Y = _data(rows, widths)
    res = []
    for fuse in (True, False):
        _, ar, eng = _engine(widths, rows, "cuda", HipOps("cuda"), lr=1e-3, momentum=0.9,
                             fuse_sgd=fuse, rowband=True, monkeypatch=monkeypatch)
        assert eng.rowband and eng.uses_rowband_split(rows) == split
        eng.load_batch(X, Y)
        eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
        for _ in range(3):
            eng.step()
        eng.synchronize()
        res.append((ar.master.clone(), ar.momentum.clone(), ar.shadow.clone(), eng.loss()))
    for a, b in zip(res[0][:3], res[1][:3]):
        assert torch.equal(a, b)
    assert res[0][3] == res[1][3]


@pytest.mark.parametrize("widths,rows,fuse", [([512, 512, 512, 512, 1], 8192, True),
                                              ([512, 512, 512, 512, 1], 8192, False),
                                              ([256, 512, 512, 512, 1], 3000, True),
                                              ([128, 384, 384, 1], 777, True),
                                              ([1024, 512, 512, 1], 4096, False),
                                              ([512, 256, 1], 64, True)])
def test_rowband_in_launch_fixup_is_bitwise_equal_to_combine_launch(widths, rows, fuse, monkeypatch):
    """The split-K combine inside the weight-gradient launch (the last split of each tile sums
    the slabs and applies the update, wgrad_multi_fix) against the separate combine launch
    (slab_multi): three steps, bitwise-equal master, momentum, shadow, weight images and loss --
    with the fused update (one rank) and with gradients + the optimizer pass."""
    from nnmpi_amd import native
    from nnmpi_amd.ops.hip_ops import HipOps
    lib = native.lib()
    if not lib.experiments_built():
        # production library: the in-launch fixup is not compiled in, its switch refuses
        with pytest.raises(RuntimeError, match="experiments build only"):
            lib.set_rb_fixup(1)
        pytest.skip("in-launch fixup: experiments library only (NNMPI_BUILD_EXPERIMENTS=1)")
    X, Y = _data(rows, widths)
    res = []
    monkeypatch.setenv("NNMPI_ROWBAND_MIN_ROWS", "1")
    try:
        for fix in (1, 0):
            assert lib.set_rb_fixup(fix)
            _, ar, eng = _engine(widths, rows, "cuda", HipOps("cuda"), lr=1e-3, momentum=0.9,
                                 fuse_sgd=fuse, rowband=True, monkeypatch=monkeypatch)
            assert eng.rowband and eng.uses_rowband(rows)
            eng.load_batch(X, Y)
            eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
            for _ in range(3):
                eng.step()
            eng.synchronize()
            res.append((ar.master.clone(), ar.momentum.clone(), ar.shadow.clone(),
                        eng._rb_buf.clone(), eng.loss()))
    finally:
        lib.set_rb_fixup(-1)
    for a, b in zip(res[0][:4], res[1][:4]):
        assert torch.equal(a, b)
    assert res[0][4] == res[1][4]


@pytest.mark.parametrize("widths,rows", [([512, 512, 512, 512, 1], 8192), ([256, 512, 512, 512, 1], 3000),
                                         ([128, 384, 384, 1], 6500)])
def test_rowband_half_width_wgrad_tile_is_bitwise_equal(widths, rows, monkeypatch):
    """The 128 x 64 weight-gradient tile (NNMPI_WGM_TILE=1, two blocks per CU) against the
    128 x 128 tile: same K split, same accumulation order -- bitwise-equal parameters, momentum
    and images after three fused-update steps."""
    from nnmpi_amd import native
    from nnmpi_amd.ops.hip_ops import HipOps
    lib = native.lib()
    if not lib.experiments_built():
        with pytest.raises(RuntimeError, match="experiments build only"):
            lib.set_wgm_tile(1)
        pytest.skip("half-width tile: experiments library only (NNMPI_BUILD_EXPERIMENTS=1)")
    X, Y = _data(rows, widths)
    res = []
    monkeypatch.setenv("NNMPI_ROWBAND_MIN_ROWS", "1")
    try:
        for tile in (1, 0):
            assert lib.set_wgm_tile(tile)
            _, ar, eng = _engine(widths, rows, "cuda", HipOps("cuda"), lr=1e-3, momentum=0.9,
                                 fuse_sgd=True, rowband=True, monkeypatch=monkeypatch)
            eng.load_batch(X, Y)
            eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
            for _ in range(3):
                eng.step()
            eng.synchronize()
            res.append((ar.master.clone(), ar.momentum.clone(), eng._rb_buf.clone(), eng.loss()))
    finally:
        lib.set_wgm_tile(-1)
    for a, b in zip(res[0][:3], res[1][:3]):
        assert torch.equal(a, b)
    assert res[0][3] == res[1][3]


@pytest.mark.parametrize("widths,rows", [([512, 512, 512, 512, 1], 8192), ([256, 256, 256, 1], 8192),
                                         ([768, 1024, 1024, 1], 8192), ([384, 384, 384, 1], 8192),
                                         ([512, 512, 512, 512, 1], 1024), ([256, 512, 512, 1], 2000)])
def test_rowband_fused_update_writes_the_weight_images(widths, rows, monkeypatch):
    """The combines that apply the update also rewrite the v2 weight images (the forward image
    directly, the transposed dgrad image staged through LDS where a block holds whole rows):
    after a few steps they equal a fresh pack of the new bf16 weights, bit for bit.  At 1,024 /
    2,000 rows: the small-batch path's weight-gradient epilogue (wgrad_small) writes them."""
    from nnmpi_amd.ops.hip_ops import HipOps
    if rows < 6144:
        monkeypatch.setenv("NNMPI_ROWBAND_MIN_ROWS", "6144")
    X, Y = _data(rows, widths)
    ops = HipOps("cuda")
    _, ar, eng = _engine(widths, rows, "cuda", ops, lr=1e-3, momentum=0.9, fuse_sgd=True,
                         rowband=True, monkeypatch=monkeypatch)
    assert eng.rowband and eng.rb_version == 2
    assert eng.uses_rowband_split(rows) == (rows < 6144)
    eng.load_batch(X, Y)
    eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
    for _ in range(3):
        eng.step()
    eng.synchronize()
    nh = len(widths) - 2
    buf, fresh = ops.rowband_packed(widths[1], widths[0], nh, "cuda")
    ops.rowband_pack([ar.compute_weight(i) for i in range(nh)], fresh)
    torch.cuda.synchronize()
    for l, ((pf, pd), (qf, qd)) in enumerate(zip(eng.rb_packed, fresh)):
        assert torch.equal(pf, qf), f"forward image of layer {l}"
        if pd is not None:
            assert torch.equal(pd, qd), f"dgrad image of layer {l}"


@pytest.mark.parametrize("widths,rows,fuse", [([512, 512, 512, 512, 1], 8192, False),
                                              ([256, 512, 512, 512, 1], 1000, False),
                                              ([512] * 5 + [1], 2000, False),
                                              ([768, 768, 768, 1], 6144, False)])
def test_rowband_optimizer_pass_writes_the_weight_images(widths, rows, fuse, monkeypatch):
    """The optimizer pass of the multi-rank row-band step (gradients first, then ops.sgd with
    the images: here fuse_sgd=False at one rank runs exactly that pass) refreshes the v2 images
    through the tiled kernel (optim.hip sgd_tiles_kernel): after three steps the images equal a
    fresh pack of the new bf16 weights, and master / momentum / shadow / images / loss are bitwise
    those of the element-wise pass (NNMPI_SGD_TILES=0)."""
    from nnmpi_amd.ops.hip_ops import HipOps
    if rows < 6144:
        monkeypatch.setenv("NNMPI_ROWBAND_MIN_ROWS", "6144")
    X, Y = _data(rows, widths)
    res = []
    for tiles in ("1", "0"):
        monkeypatch.setenv("NNMPI_SGD_TILES", tiles)
        from nnmpi_amd import native
        native.lib().set_sgd_tiles(-1)
        ops = HipOps("cuda")
        _, ar, eng = _engine(widths, rows, "cuda", ops, lr=1e-3, momentum=0.9, fuse_sgd=fuse,
                             rowband=True, monkeypatch=monkeypatch)
        assert eng.rowband and eng.rb_version == 2
        eng.load_batch(X, Y)
        eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
        for _ in range(3):
            eng.step()
        eng.synchronize()
        nh = len(widths) - 2
        buf, fresh = ops.rowband_packed(widths[1], widths[0], nh, "cuda")
        ops.rowband_pack([ar.compute_weight(i) for i in range(nh)], fresh)
        torch.cuda.synchronize()
        assert torch.equal(eng._rb_buf, buf), f"images (tiles={tiles}) differ from a fresh pack"
        res.append((ar.master.clone(), ar.momentum.clone(), ar.shadow.clone(), eng._rb_buf.clone(),
                    eng.loss()))
    native.lib().set_sgd_tiles(-1)
    for a, b in zip(res[0][:4], res[1][:4]):
        assert torch.equal(a, b)
    assert res[0][4] == res[1][4]


@pytest.mark.parametrize("rows", [8192, 1024, 3000])
def test_rowband_graph_replay_is_bitwise_equal_to_eager(rows, monkeypatch):
    """Graph replay vs eager, 4 fused-update steps, bitwise (at 1,024 / 3,000 rows the
    column-split kernel: its per-band counters reset themselves, so replays see zero)."""
    from nnmpi_amd.engine.arena import Arena
    from nnmpi_amd.engine.engine import MLPEngine
    from nnmpi_amd.models.mlp import MLPSpec, reference_init
    from nnmpi_amd.ops.hip_ops import HipOps
    from nnmpi_amd.parallel.sync import NoSync
    monkeypatch.setenv("NNMPI_ROWBAND", "1")
    monkeypatch.setenv("NNMPI_ROWBAND_MIN_ROWS", "6144")   # (the production threshold)
    widths = [512, 512, 512, 512, 1]
    X, Y = _data(rows, widths)
    spec = MLPSpec(tuple(widths), "relu", "mse")
    out = []
    for graph in (False, True):
        ar = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], "cuda",
                   shadow_dtype=torch.bfloat16)
        ar.bind_model(reference_init(widths, "relu", seed=5))
        eng = MLPEngine(spec, ar, HipOps("cuda"), NoSync(ar), device="cuda", dtype=torch.bfloat16,
                        rows_capacity=rows, lr=1e-3, momentum=0.9, use_graph=graph)
        assert eng.rowband and eng.uses_rowband(rows)
        assert eng.uses_rowband_split(rows) == (rows < 6144)
        eng.load_batch(X, Y)
        eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
        for _ in range(4):
            eng.step()
        eng.synchronize()
        out.append((ar.master.clone(), eng.loss()))
    assert torch.equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]


def test_bench_default_proxy_step_runs_the_rowband_schedule():
    """The driver's default 1-GPU bench (the BASELINE proxy) times the row-band step."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "6",
                        "--warmup", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["config"]["schedule"] == "rowband"
    assert d["replicas_bitwise_equal"] is True and d["final_loss"] == d["final_loss"]


def test_small_batches_pick_the_split_kernel_or_the_grouped_schedule(monkeypatch):
    """Below NNMPI_ROWBAND_MIN_ROWS (default 4,097 for 512-wide hidden layers, 6,144 otherwise)
    the band kernel is not taken (a band's passes cost the same however few bands there are): the
    512-wide proxy's small batches (<= 4,096 rows) run the column-split kernel and 4,097 rows up
    the band kernel (5,000 rows: no grouped schedule left, profiles/r6_rowband_threshold.txt),
    other widths' small batches the grouped schedule; one engine switches between the kernels by
    batch size."""
    from nnmpi_amd.ops.hip_ops import HipOps
    monkeypatch.delenv("NNMPI_ROWBAND_MIN_ROWS", raising=False)
    widths = [512, 512, 512, 512, 1]
    _, _, eng = _engine(widths, 8192, "cuda", HipOps("cuda"), rowband=True, monkeypatch=monkeypatch)
    X, Y = _data(8192, widths)
    seen = []
    for rows, split, name in ((1024, True, "rowband"), (5000, False, "rowband"),
                              (8192, False, "rowband"), (2048, True, "rowband")):
        eng.load_batch(X[:rows], Y[:rows])
        assert eng.uses_rowband_split() == split and eng.schedule_name() == name, rows
        eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
        eng.step()
        seen.append(eng.loss())
    assert all(v == v for v in seen)
    _, _, e256 = _engine([256, 256, 256, 256, 1], 1024, "cuda", HipOps("cuda"), rowband=True,
                         monkeypatch=monkeypatch)
    X2, Y2 = _data(1024, [256, 256, 256, 256, 1])
    e256.load_batch(X2, Y2)
    assert not e256.uses_rowband() and e256.schedule_name() == "grouped"



def test_rowband_checkpoint_resume_is_exact(tmp_path):
    """Checkpoint / resume through the row-band schedule: 3 epochs + resume to 6 == 6 epochs bit
    for bit (the resumed arena bumps Arena.version, so the v2 weight images are rebuilt from the
    loaded weights before the first resumed step; the momentum is restored by name)."""
    from nnmpi_amd.engine import trainer
    from nnmpi_amd.utils.config import TrainConfig
    base = dict(device="cuda", print_rank="none", widths=[512, 512, 512, 512, 1], n_features=512,
                n_samples=8192, dtype="bf16", lr=1e-4, data_gen="device", data_dist="local",
                scaling="none")
    ck = str(tmp_path / "rb.pt")
    full = trainer.run_worker(TrainConfig(nepochs=6, **base))
    trainer.run_worker(TrainConfig(nepochs=3, checkpoint=ck, **base))
    res = trainer.run_worker(TrainConfig(nepochs=6, resume=ck, **base))
    assert full.schedule["rowband"] and res.schedule["rowband"]
    assert torch.equal(res.final_params, full.final_params)
    assert res.losses[-3:] == full.losses[-3:]
