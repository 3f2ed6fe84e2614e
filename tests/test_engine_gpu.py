"""End-to-end engine tests on one MI355X: golden parity, GPU vs CPU oracle, graph replay."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"

from test_golden import GOLDEN_LOSSES, GOLDEN_PARAMS  # noqa: E402

import nnmpi_amd  # noqa: E402
from nnmpi_amd.engine import trainer  # noqa: E402
from nnmpi_amd.utils.config import TrainConfig  # noqa: E402


def test_reference_config_on_gpu_matches_golden():
    res = trainer.run_worker(TrainConfig(device="cuda", print_rank="none"))
    assert res.losses == pytest.approx(GOLDEN_LOSSES[1][0], rel=1e-5)
    assert torch.allclose(res.final_params, torch.tensor(GOLDEN_PARAMS[1]), atol=5e-6)


@pytest.mark.parametrize("graph", [False, True])
def test_reference_config_graph_modes(graph):
    res = trainer.run_worker(TrainConfig(device="cuda", print_rank="none", graph=graph, nepochs=6))
    ref = trainer.run_worker(TrainConfig(device="cpu", print_rank="none", nepochs=6))
    assert res.losses == pytest.approx(ref.losses, rel=1e-5)


def _cfg(**kw):
    base = dict(widths=[256, 256, 256, 1], n_features=256, n_samples=2048, dtype="bf16",
                print_rank="none", nepochs=4, lr=1e-3, data_gen="device", data_dist="local",
                scaling="none")
    base.update(kw)
    return TrainConfig(**base)


def test_bf16_engine_vs_cpu_oracle():
    gpu = trainer.run_worker(_cfg(device="cuda"))
    # CPU oracle with the same bf16 rounding contract; same data (generated on the GPU then moved)
    import nnmpi_amd.engine.trainer as tr
    orig = tr.build_shard

    def shard_from_gpu(j):
        jj = type("J", (), {})()
        jj.__dict__.update(j.__dict__)
        jj.device = torch.device("cuda")
        X, Y, lab, part = orig(jj)
        return X.cpu(), (Y.cpu() if Y is not None else None), lab, part
    tr.build_shard = shard_from_gpu
    try:
        cpu = trainer.run_worker(_cfg(device="cpu"))
    finally:
        tr.build_shard = orig
    assert gpu.losses == pytest.approx(cpu.losses, rel=3e-2)
    assert torch.allclose(gpu.final_params, cpu.final_params, atol=3e-3, rtol=3e-2)


def test_graph_replay_is_bitwise_equal_to_eager():
    a = trainer.run_worker(_cfg(device="cuda", graph=True, nepochs=5))
    b = trainer.run_worker(_cfg(device="cuda", graph=False, nepochs=5))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_fp32_generic_gemm_path_vs_cpu():
    kw = dict(widths=[64, 48, 32, 1], n_features=64, n_samples=512, dtype="fp32", nepochs=3,
              print_rank="none")
    gpu = trainer.run_worker(TrainConfig(device="cuda", **kw))
    cpu = trainer.run_worker(TrainConfig(device="cpu", **kw))
    assert gpu.losses == pytest.approx(cpu.losses, rel=1e-4)
    assert torch.allclose(gpu.final_params, cpu.final_params, atol=1e-5, rtol=1e-4)


def test_mnist_shape_xent_trains():
    cfg = TrainConfig(device="cuda", widths=[784, 1024, 1024, 10], n_features=784, loss="xent",
                      n_samples=4096, dtype="bf16", nepochs=20, lr=0.05, print_rank="none",
                      data_gen="device", data_dist="local")
    res = trainer.run_worker(cfg)
    assert res.losses[-1] < res.losses[0]


def test_overlapped_schedule_is_bitwise_equal_to_sequential():
    a = trainer.run_worker(_cfg(device="cuda", overlap=True, nepochs=5))
    b = trainer.run_worker(_cfg(device="cuda", overlap=False, nepochs=5))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_overlap_with_small_buckets_and_mse_head():
    a = trainer.run_worker(_cfg(device="cuda", overlap=True, bucket_mb=0.01, nepochs=4))
    b = trainer.run_worker(_cfg(device="cuda", overlap=False, bucket_mb=64, nepochs=4))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_fused_optimizer_path_is_bitwise_equal():
    """Single-rank fast path (SGD applied inside the split-K reducers) == separate SGD pass."""
    import nnmpi_amd.engine.engine as eng_mod
    a = trainer.run_worker(_cfg(device="cuda", nepochs=5))
    orig = eng_mod.MLPEngine.__init__

    def no_fuse(self, *args, **kw):
        kw["fuse_sgd"] = False
        orig(self, *args, **kw)
    eng_mod.MLPEngine.__init__ = no_fuse
    try:
        b = trainer.run_worker(_cfg(device="cuda", nepochs=5))
    finally:
        eng_mod.MLPEngine.__init__ = orig
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_native_rccl_path_single_rank_matches_local():
    """1-rank RCCL communicator: bucketed all-reduce on the comm stream + per-bucket SGD
    (captured in the step graph) must reproduce the communication-free run bitwise."""
    a = trainer.run_worker(_cfg(device="cuda", comm="native", nepochs=5))
    b = trainer.run_worker(_cfg(device="cuda", comm="none", nepochs=5))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_native_rccl_path_mnist_xent():
    cfg = dict(widths=[784, 1024, 1024, 10], n_features=784, loss="xent", n_samples=2048,
               dtype="bf16", nepochs=4, lr=0.05, print_rank="none", data_gen="device",
               data_dist="local")
    a = trainer.run_worker(TrainConfig(device="cuda", comm="native", **cfg))
    b = trainer.run_worker(TrainConfig(device="cuda", comm="none", **cfg))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def _run_ungrouped(cfg):
    import nnmpi_amd.engine.engine as eng_mod
    orig = eng_mod.MLPEngine.__init__

    def no_group(self, *args, **kw):
        kw["grouped"] = False
        orig(self, *args, **kw)
    eng_mod.MLPEngine.__init__ = no_group
    try:
        return trainer.run_worker(cfg)
    finally:
        eng_mod.MLPEngine.__init__ = orig


@pytest.mark.parametrize("comm", ["none", "native"])
def test_grouped_backward_is_bitwise_equal(comm):
    """dgrad_i + wgrad_i + combine_{i+1} in one launch == separate launches, bit for bit
    (fused-SGD single-rank path and the inline-RCCL path)."""
    a = trainer.run_worker(_cfg(device="cuda", comm=comm, nepochs=5))
    b = _run_ungrouped(_cfg(device="cuda", comm=comm, nepochs=5))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


@pytest.mark.parametrize("rows", [1024, 16])
def test_grouped_backward_small_batches_bitwise_equal(rows):
    """Small per-rank batches (strong-scaling shards: 8192 / 8 rows) run the grouped backward
    with 128x128 tiles where the standalone dgrad takes 64x64: same accumulation order, so bit
    for bit the separate launches."""
    kw = dict(device="cuda", widths=[512, 512, 512, 1], n_features=512, n_samples=rows,
              lr=1e-5, nepochs=5)
    a = trainer.run_worker(_cfg(**kw))
    b = _run_ungrouped(_cfg(**kw))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_grouped_backward_xent_head_bitwise_equal():
    cfg = TrainConfig(device="cuda", widths=[784, 1024, 1024, 10], n_features=784, loss="xent",
                      n_samples=2048, dtype="bf16", nepochs=4, lr=0.05, print_rank="none",
                      data_gen="device", data_dist="local")
    a = trainer.run_worker(cfg)
    b = _run_ungrouped(cfg)
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


@pytest.mark.parametrize("mode", ["inline", "overlap"])
def test_native_rccl_bf16_gradient_payload(mode):
    """bf16 all-reduce payload through the native communicator (cast kernels + ncclBfloat16),
    inline and on the comm stream: tracks the fp32-payload run within bf16 rounding."""
    a = trainer.run_worker(_cfg(device="cuda", comm="native", grad_dtype="bf16", comm_mode=mode,
                                nepochs=5))
    b = trainer.run_worker(_cfg(device="cuda", comm="native", comm_mode=mode, nepochs=5))
    assert all(x == x for x in a.losses)
    torch.testing.assert_close(a.final_params, b.final_params, rtol=2e-2, atol=1e-3)


def test_profile_steps_gpu_breakdown():
    res = trainer.run_worker(_cfg(device="cuda", nepochs=3, profile_steps=True))
    assert {"start->fwd", "fwd->head", "head->bwd"} <= set(res.phase_ms)
    assert res.phase_ms["start->fwd"] > 0


def test_multi_step_graph_equals_single_steps():
    """run_steps(n, chunk) replays graphs of `chunk` whole steps: bitwise equal to n step()s."""
    outs = []
    for chunk in (1, 3):
        import torch as _t
        from nnmpi_amd.engine.arena import Arena
        from nnmpi_amd.engine.engine import MLPEngine
        from nnmpi_amd.models.mlp import MLPSpec, reference_init
        from nnmpi_amd.ops.hip_ops import HipOps
        from nnmpi_amd.parallel.sync import NoSync
        from nnmpi_amd.data import synth
        widths = [256, 256, 256, 1]
        spec = MLPSpec(tuple(widths), "relu", "mse")
        ar = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], "cuda",
                   shadow_dtype=_t.bfloat16)
        ar.bind_model(reference_init(widths, "relu", seed=0))
        eng = MLPEngine(spec, ar, HipOps("cuda"), NoSync(ar), device="cuda", dtype=_t.bfloat16,
                        rows_capacity=1024, lr=1e-4, momentum=0.9)
        X, Y = synth.chunked_regression(0, 1024, 256, device="cuda")
        eng.load_batch(X.to(_t.bfloat16), Y)
        eng.set_scales(1 / 1024, 1 / 1024, 1.0)
        eng.run_steps(10, chunk)
        eng.synchronize()
        outs.append(ar.master.clone())
        assert eng.steps_done == 10
    assert _t.equal(outs[0], outs[1])


def _cfg512(**kw):
    """Proxy-sized shapes (8192 x 512): the 128x128-tile forward and the grouped backward."""
    return _cfg(device="cuda", widths=[512, 512, 512, 1], n_features=512, n_samples=8192,
                lr=1e-5, **kw)


@pytest.mark.parametrize("mode", [1, 2])
def test_grouped_backward_async_lds_reads_bitwise_equal(mode):
    """Grouped backward with asm transposed LDS reads (explicit lgkmcnt, DMA ring kept in
    flight) == the compiler-scheduled reads, bit for bit."""
    from nnmpi_amd import native
    lib = native.lib()
    try:
        lib.set_group_async(0)
        a = trainer.run_worker(_cfg512(nepochs=5))
        lib.set_group_async(mode)
        b = trainer.run_worker(_cfg512(nepochs=5))
    finally:
        lib.set_group_async(-1)
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


@pytest.mark.parametrize("variant", [1, 2, 5, 6, 8, 10, 11, 12, 13])
def test_forward_variants_bitwise_equal(variant):
    """Every forward main-loop variant accumulates each output in the same k order."""
    from nnmpi_amd import native
    lib = native.lib()
    try:
        lib.set_fwd_variant(0)
        a = trainer.run_worker(_cfg512(nepochs=3))
        lib.set_fwd_variant(variant)
        b = trainer.run_worker(_cfg512(nepochs=3))
    finally:
        lib.set_fwd_variant(-1)
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_native_root_sync_single_rank_matches_local():
    """--sync root over RCCL (ncclReduce to rank 0 + ncclBroadcast, the reference's pattern)."""
    a = trainer.run_worker(_cfg(device="cuda", comm="native", sync="root", nepochs=4))
    b = trainer.run_worker(_cfg(device="cuda", comm="none", nepochs=4))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_native_sharded_optimizer_single_rank_matches_local():
    """ZeRO-1 through the native communicator (in-place ncclReduceScatter, owner SGD, in-place
    bf16 ncclAllGather, final fp32 gather) == the communication-free run."""
    a = trainer.run_worker(_cfg(device="cuda", comm="native", shard_optimizer=True, nepochs=4))
    b = trainer.run_worker(_cfg(device="cuda", comm="none", nepochs=4))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_native_scatterv_single_rank():
    """RcclComm.scatterv (grouped ncclSend/ncclRecv; the root's own chunk is a device copy)."""
    from nnmpi_amd import native
    lib = native.lib()
    comm = native.make_comm(lib.rccl_unique_id(), 1, 0, torch.cuda.current_device())
    src = torch.arange(30, dtype=torch.float64, device="cuda")
    dst = torch.zeros(12, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    comm.scatterv(src.data_ptr(), [12], [6], dst.data_ptr(), 2, 0, int(s.cuda_stream))
    s.synchronize()
    assert torch.equal(dst, src[6:18])


def test_tiny_fused_optimizer_is_bitwise_equal():
    """Reference 2-3-1 config: the one-block tiny kernel applying SGD itself (one launch per
    step) == tiny kernel + separate optimizer pass."""
    import nnmpi_amd.engine.engine as eng_mod
    a = trainer.run_worker(TrainConfig(device="cuda", print_rank="none", nepochs=8))
    orig = eng_mod.MLPEngine.__init__

    def no_fuse(self, *args, **kw):
        kw["fuse_sgd"] = False
        orig(self, *args, **kw)
    eng_mod.MLPEngine.__init__ = no_fuse
    try:
        b = trainer.run_worker(TrainConfig(device="cuda", print_rank="none", nepochs=8))
    finally:
        eng_mod.MLPEngine.__init__ = orig
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_unsplit_wgrad_epilogue_optimizer_is_bitwise_equal():
    """Single rank, weight gradients without split-K (the 8192-wide case; forced here): the SGD
    update applied in the wgrad GEMM epilogue == gradient store + separate optimizer pass."""
    from nnmpi_amd import native
    import nnmpi_amd.engine.engine as eng_mod
    lib = native.lib()
    orig = eng_mod.MLPEngine.__init__

    def no_group(self, *args, **kw):
        kw["grouped"] = False
        orig(self, *args, **kw)

    def no_fuse(self, *args, **kw):
        kw["grouped"] = False
        kw["fuse_sgd"] = False
        orig(self, *args, **kw)
    try:
        lib.set_wgrad_splits(1)
        eng_mod.MLPEngine.__init__ = no_group
        a = trainer.run_worker(_cfg(device="cuda", nepochs=4))
        eng_mod.MLPEngine.__init__ = no_fuse
        b = trainer.run_worker(_cfg(device="cuda", nepochs=4))
    finally:
        lib.set_wgrad_splits(0)
        eng_mod.MLPEngine.__init__ = orig
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_validation_split_gpu_matches_cpu():
    """Forward-only evaluation on GPU (tiny fp32 kernel, and the bf16 GEMM + head path)."""
    a = trainer.run_worker(TrainConfig(device="cuda", print_rank="none", val_fraction=0.25))
    b = trainer.run_worker(TrainConfig(device="cpu", print_rank="none", val_fraction=0.25))
    assert a.val_losses == pytest.approx(b.val_losses, rel=1e-5)
    c = trainer.run_worker(_cfg(device="cuda", val_fraction=0.2, nepochs=3))
    assert len(c.val_losses) == 3 and all(v == v for v in c.val_losses)
    assert c.losses[-1] < c.losses[0]


def test_gather_rows_kernel():
    from nnmpi_amd.ops.hip_ops import HipOps
    ops = HipOps()
    g = torch.Generator(device="cpu").manual_seed(3)
    idx = torch.randint(0, 100, (77,), generator=g).to(DEV)
    for src in (torch.randn(100, 37, device=DEV), torch.randn(100, 64, device=DEV).to(torch.bfloat16),
                torch.arange(100, device=DEV)):
        dst = torch.zeros((80,) + tuple(src.shape[1:]), dtype=src.dtype, device=DEV)
        ops.gather_rows(src, idx, dst)
        assert torch.equal(dst[:77], src[idx])


def test_minibatch_training_gpu_matches_cpu():
    kw = dict(widths=[64, 48, 32, 1], n_features=64, n_samples=512, dtype="fp32", nepochs=2,
              print_rank="none", batch_size=96)
    gpu = trainer.run_worker(TrainConfig(device="cuda", **kw))
    cpu = trainer.run_worker(TrainConfig(device="cpu", **kw))
    assert gpu.steps == cpu.steps == 2 * 6
    assert gpu.losses == pytest.approx(cpu.losses, rel=1e-4)
    assert torch.allclose(gpu.final_params, cpu.final_params, atol=1e-5, rtol=1e-4)


def test_grad_accum_gpu_matches_cpu_and_single_batch():
    """Accumulated micro-batches on the GPU (fp32 GEMMs, then the tiny kernel with its in-kernel
    SGD switched off) == the CPU oracle, and == one batch of the same rows."""
    kw = dict(widths=[64, 48, 32, 1], n_features=64, n_samples=512, dtype="fp32", nepochs=2,
              print_rank="none", batch_size=64, grad_accum=3)
    gpu = trainer.run_worker(TrainConfig(device="cuda", **kw))
    cpu = trainer.run_worker(TrainConfig(device="cpu", **kw))
    assert gpu.steps == cpu.steps == 2 * 3
    assert gpu.losses == pytest.approx(cpu.losses, rel=1e-4)
    assert torch.allclose(gpu.final_params, cpu.final_params, atol=1e-5, rtol=1e-4)
    one = trainer.run_worker(TrainConfig(device="cuda", **dict(kw, batch_size=192, grad_accum=1)))
    assert torch.allclose(gpu.final_params, one.final_params, atol=1e-5, rtol=1e-4)
    t = dict(print_rank="none", nepochs=4)
    a = trainer.run_worker(TrainConfig(device="cuda", grad_accum=2, **t))
    b = trainer.run_worker(TrainConfig(device="cpu", grad_accum=2, **t))
    assert a.losses == pytest.approx(b.losses, rel=1e-5)
    c = trainer.run_worker(_cfg(device="cuda", nepochs=3, grad_accum=2))
    assert c.losses[-1] < c.losses[0]


@pytest.mark.parametrize("grouped", [True, False])
def test_xent_head_optimizer_fusion_is_bitwise_equal(grouped):
    """Multi-output head: SGD applied in the head weight-gradient combine (deferred into the
    grouped backward launch, or run right after the head) == a separate SGD pass."""
    import nnmpi_amd.engine.engine as eng_mod
    cfg = TrainConfig(device="cuda", widths=[784, 1024, 1024, 10], n_features=784, loss="xent",
                      n_samples=2048, dtype="bf16", nepochs=4, lr=0.05, print_rank="none",
                      data_gen="device", data_dist="local")
    orig = eng_mod.MLPEngine.__init__

    def patched(fuse):
        def init(self, *args, **kw):
            kw["fuse_sgd"] = fuse
            kw["grouped"] = grouped
            orig(self, *args, **kw)
        return init
    try:
        eng_mod.MLPEngine.__init__ = patched(True)
        a = trainer.run_worker(cfg)
        eng_mod.MLPEngine.__init__ = patched(False)
        b = trainer.run_worker(cfg)
    finally:
        eng_mod.MLPEngine.__init__ = orig
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def _wide_cfg(**kw):
    base = dict(widths=[8192, 8192, 8192, 1], n_features=8192, n_samples=512, dtype="bf16",
                nepochs=3, lr=1e-4, data_gen="device", data_dist="local", scaling="none",
                print_rank="none", device="cuda")
    base.update(kw)
    return TrainConfig(**base)


@pytest.mark.parametrize("width,rows", [(4096, 4096), (8192, 512)])
def test_wide_pair_launches_bitwise_equal(width, rows):
    """Single rank, 256x256-tile layers: wgrad_i + SGD epilogue beside dgrad_{i-1} (and the last
    two weight gradients together) in one interleaved launch each == the separate launches.
    4096 rows: both pair kinds; 512 rows: the dgrads are too small to pair (fallback) and only
    the last two weight gradients share a launch."""
    from nnmpi_amd import native
    lib = native.lib()
    if not lib.experiments_built():
        # production build: the pair kernel is not linked and every pair is refused
        assert not lib.wide_pair_wgrad_ok(rows, width, width)
        pytest.skip("experiment kernels not built (NNMPI_BUILD_EXPERIMENTS=1)")
    cfg = _wide_cfg(widths=[width] * 4 + [1], n_features=width, n_samples=rows)
    try:
        lib.set_wide_pair(1)
        a = trainer.run_worker(cfg)
        lib.set_wide_pair(0)
        b = trainer.run_worker(cfg)
    finally:
        lib.set_wide_pair(-1)
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)
    assert a.losses[-1] == a.losses[-1]


@pytest.mark.parametrize("width,rows", [(4096, 4096), (4000, 1000)])
def test_pp256_one_half_per_phase_bitwise_equal(width, rows):
    """The 256x256 kernel with one DMA half per phase (set_pp256_order 2 / 3) gives the same bits
    as the default 1/0/2/1 placement for the forward, dgrad and weight gradient (full and ragged
    tiles): only the issue point of B0(t+2) and the counted waits move."""
    from nnmpi_amd import native
    lib = native.lib()
    cfg = _wide_cfg(widths=[width] * 4 + [1], n_features=width, n_samples=rows)
    out = []
    try:
        for orders in ((0, 0, 1), (2, 2, 3)):
            for epi, idx in enumerate(orders):
                lib.set_pp256_order(epi, idx)
            out.append(trainer.run_worker(cfg))
    finally:
        for epi, idx in enumerate((0, 0, 1)):
            lib.set_pp256_order(epi, idx)
    assert out[0].losses == out[1].losses
    assert torch.equal(out[0].final_params, out[1].final_params)


@pytest.mark.parametrize("width,rows", [(4096, 4096), (4096, 600), (4000, 1000)])
def test_wide_sgd_epilogue_forms_bitwise_equal(width, rows):
    """Single rank, 256x256 weight-gradient tiles with the SGD update in the epilogue: the
    LDS-staged row form (default), the per-fragment form and the batched-fragment form give
    identical parameters.  600 rows: partial dgrad/forward tiles; 4000 wide: the edge weight
    tiles are partial, so interior tiles take the LDS form and edge tiles fall back to the
    fragment form inside the same launch."""
    from nnmpi_amd import native
    lib = native.lib()
    cfg = _wide_cfg(widths=[width] * 4 + [1], n_features=width, n_samples=rows)
    out = []
    try:
        for form in (0, 1, 2):
            lib.set_sgd_epilogue(form)
            out.append(trainer.run_worker(cfg))
    finally:
        lib.set_sgd_epilogue(-1)
    for r in out[1:]:
        assert r.losses == out[0].losses
        assert torch.equal(r.final_params, out[0].final_params)


@pytest.mark.parametrize("width,rows", [(4096, 4096), (4000, 1000)])
def test_wide_staged_forward_epilogue_bitwise_equal(width, rows):
    """256x256 forward tiles: bias + activation staged through LDS with row stores == the
    fragment stores (4000 wide / 1000 rows: partial edge tiles keep the fragment form)."""
    from nnmpi_amd import native
    lib = native.lib()
    cfg = _wide_cfg(widths=[width] * 4 + [1], n_features=width, n_samples=rows)
    out = []
    try:
        for on in (1, 0):
            lib.set_stage_epi(on)
            out.append(trainer.run_worker(cfg))
    finally:
        lib.set_stage_epi(-1)
    assert out[0].losses == out[1].losses
    assert torch.equal(out[0].final_params, out[1].final_params)


def test_wide_chunked_buckets_overlap_bitwise_equal():
    """8192-wide layers cut into 4 output-row chunk buckets: each chunk's weight gradient is
    its own launch, its all-reduce starts behind it on the comm stream, its SGD runs on the
    update stream -- bitwise equal to the communication-free run (SGD fused in the epilogue)."""
    a = trainer.run_worker(_wide_cfg(comm="native", comm_mode="overlap", bucket_mb=16,
                                     grad_dtype="fp32"))
    b = trainer.run_worker(_wide_cfg(comm="none"))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_wide_chunked_bf16_payload_written_by_wgrad_bitwise_equal():
    """bf16 payload, overlapped: the chunk weight gradients store bf16 straight into the
    all-reduce buffer (no fp32 gradient, no cast pass) and the SGD reads it -- bitwise equal to
    the inline bf16 path (fp32 gradient -> cast -> all-reduce -> cast back -> SGD)."""
    a = trainer.run_worker(_wide_cfg(comm="native", comm_mode="overlap", bucket_mb=16,
                                     grad_dtype="bf16"))
    b = trainer.run_worker(_wide_cfg(comm="native", comm_mode="inline", grad_dtype="bf16"))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


def test_grouped_backward_with_comm_overlap_bitwise_equal():
    """Grouped backward (dgrad + wgrad + combine in one launch) with per-bucket all-reduce on
    the comm stream and SGD on the update stream == the fused single-rank path."""
    a = trainer.run_worker(_cfg512(comm="native", comm_mode="overlap", nepochs=4))
    b = trainer.run_worker(_cfg512(comm="none", nepochs=4))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


@pytest.mark.parametrize("widths,loss", [([512, 256, 100], "xent"), ([8192, 256, 10], "xent"),
                                         ([256, 256, 40], "mse")])
def test_general_head_engine_vs_cpu_oracle(widths, loss):
    """Output layers beyond the skinny head kernels train end to end (grouped / fused
    schedules with the head's update as a separate pass) and track the CPU oracle."""
    kw = dict(widths=widths, n_features=widths[0], loss=loss, n_samples=1024, dtype="fp32",
              nepochs=3, lr=0.05 if loss == "xent" else 1e-4, print_rank="none",
              data_gen="device", data_dist="local", scaling="none")
    gpu = trainer.run_worker(TrainConfig(device="cuda", **kw))
    import nnmpi_amd.engine.trainer as tr
    orig = tr.build_shard

    def shard_from_gpu(j):
        jj = type("J", (), {})()
        jj.__dict__.update(j.__dict__)
        jj.device = torch.device("cuda")
        X, Y, lab, part = orig(jj)
        return X.cpu(), (Y.cpu() if Y is not None else None), (lab.cpu() if lab is not None
                                                               else None), part
    tr.build_shard = shard_from_gpu
    try:
        cpu = trainer.run_worker(TrainConfig(device="cpu", **kw))
    finally:
        tr.build_shard = orig
    assert gpu.losses == pytest.approx(cpu.losses, rel=1e-4)
    assert torch.allclose(gpu.final_params, cpu.final_params, atol=1e-5, rtol=1e-4)
    bf = trainer.run_worker(TrainConfig(device="cuda", **dict(kw, dtype="bf16")))
    assert bf.losses[-1] == bf.losses[-1] and bf.losses == pytest.approx(cpu.losses, rel=3e-2)


@pytest.mark.parametrize("cfg", ["bf16_512", "mnist_xent", "reference_fp32"])
def test_gpu_checkpoint_resume_is_bitwise(tmp_path, cfg):
    """Checkpoint after 3 epochs (rank-0 reference-format state_dict + momentum arena), resume
    in a fresh job and finish: bitwise equal to the uninterrupted run (bf16 compute: the shadow
    is re-derived from the fp32 master on load, the momentum-first-step flag from the step
    counter)."""
    ck = str(tmp_path / "model.pt")
    if cfg == "bf16_512":
        mk = lambda **k: _cfg512(**k)  # noqa: E731
    elif cfg == "mnist_xent":
        mk = lambda **k: TrainConfig(device="cuda", widths=[784, 1024, 1024, 10], n_features=784,  # noqa: E731
                                     loss="xent", n_samples=2048, dtype="bf16", lr=0.05,
                                     print_rank="none", data_gen="device", data_dist="local", **k)
    else:
        mk = lambda **k: TrainConfig(device="cuda", print_rank="none", **k)  # noqa: E731
    full = trainer.run_worker(mk(nepochs=5))
    trainer.run_worker(mk(nepochs=3, checkpoint=ck))
    res = trainer.run_worker(mk(nepochs=5, resume=ck))
    assert res.losses == full.losses[3:]
    assert torch.equal(res.final_params, full.final_params)
    sd = torch.load(ck, weights_only=True)
    assert all(k.startswith("layers.") for k in sd)


@pytest.mark.parametrize("widths,loss", [([512, 512, 512, 512, 1], "mse"),
                                         ([784, 1024, 1024, 10], "xent"),
                                         ([256, 256, 40], "mse")])
def test_bf16_gradients_per_layer_vs_oracle(widths, loss):
    """One backward pass from the same init and data: every layer's weight and bias gradient
    from the HIP kernels vs the PyTorch oracle with the same bf16 rounding contract, each to
    1e-2 relative norm -- tight enough that a wrong scale on any single layer / bucket (2x,
    1/P, a missing loss_scale) fails, unlike an end-of-training loss comparison."""
    from nnmpi_amd.data import synth
    from nnmpi_amd.engine.arena import Arena
    from nnmpi_amd.engine.engine import MLPEngine
    from nnmpi_amd.models.mlp import MLPSpec, reference_init
    from nnmpi_amd.ops.hip_ops import HipOps
    from nnmpi_amd.ops.torch_ops import TorchOps
    from nnmpi_amd.parallel.sync import NoSync
    rows = 1024
    spec = MLPSpec(tuple(widths), "relu", loss)
    if loss == "xent":
        X, lab = synth.chunked_classification(0, rows, widths[0], widths[-1], device="cuda")
        Y = None
    else:
        X, Y = synth.chunked_regression(0, rows, widths[0], out=widths[-1], device="cuda")
        lab = None
    grads = []
    for dev, ops in (("cuda", HipOps("cuda")), ("cpu", TorchOps("cpu"))):
        ar = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], dev,
                   shadow_dtype=torch.bfloat16)
        ar.bind_model(reference_init(widths, "relu", seed=3))
        eng = MLPEngine(spec, ar, ops, NoSync(ar), device=dev, dtype=torch.bfloat16,
                        rows_capacity=rows, lr=0.0, momentum=0.0, use_graph=False,
                        overlap=False)
        eng.load_batch(X.to(torch.bfloat16).to(dev), Y.to(dev) if Y is not None else None,
                       lab.to(dev) if lab is not None else None)
        per = widths[-1] if loss == "mse" else 1
        eng.set_scales(1.0 / (rows * per), 1.0 / (rows * per), 1.0)
        with torch.no_grad():
            if dev == "cuda":
                with torch.cuda.stream(eng.stream):
                    eng.forward_backward()
                eng.synchronize()
            else:
                eng.forward_backward()
        grads.append({li: (ar.grad_weight(li).double().cpu().clone(),
                           ar.grad_bias(li).double().cpu().clone())
                      for li in range(spec.n_layers)})
        grads[-1]["loss"] = float(eng.loss_out[0].item())
    g, r = grads
    assert g["loss"] == pytest.approx(r["loss"], rel=1e-3)
    for li in range(spec.n_layers):
        for k in range(2):
            a, b = g[li][k], r[li][k]
            rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
            assert rel < 1e-2, (li, k, rel)


def test_general_head_with_comm_overlap_bitwise_equal():
    """A head the skinny kernels do not take (its gradient is final right after the head, not
    in the first grouped launch) through the comm-overlapped grouped schedule: every bucket
    updated exactly once -- bitwise equal to the communication-free run."""
    kw = dict(widths=[512, 256, 100], n_features=512, loss="xent", n_samples=2048, dtype="bf16",
              nepochs=4, lr=0.05, print_rank="none", data_gen="device", data_dist="local",
              scaling="none")
    a = trainer.run_worker(TrainConfig(device="cuda", comm="native", comm_mode="overlap",
                                       bucket_mb=0.1, **kw))
    b = trainer.run_worker(TrainConfig(device="cuda", comm="none", **kw))
    assert a.losses == b.losses
    assert torch.equal(a.final_params, b.final_params)


@pytest.mark.parametrize("widths", [[512, 512, 512, 1], [2, 3, 1]])
def test_fast_epochs_same_output_as_per_epoch_steps(widths, capsys):
    """Full-batch epochs replayed 64 per graph with per-step losses recorded on the device print
    the same lines with the same losses, and end with the same parameters, as one replay + one
    loss readback per epoch (70 epochs: an eager first step, a 63-step and a 6-step graph)."""
    kw = dict(widths=widths, n_features=widths[0], nepochs=70, lr=1e-5, print_rank="0")
    if widths[0] == 2:
        kw = dict(nepochs=70, print_rank="0", dtype="fp32")
        a = trainer.run_worker(TrainConfig(device="cuda", **kw))
        out_a = capsys.readouterr().out
        b = trainer.run_worker(TrainConfig(device="cuda", fast_epochs=False, **kw))
    else:
        a = trainer.run_worker(_cfg(device="cuda", n_samples=4096, **kw))
        out_a = capsys.readouterr().out
        b = trainer.run_worker(_cfg(device="cuda", n_samples=4096, fast_epochs=False, **kw))
    out_b = capsys.readouterr().out
    assert a.losses == b.losses and len(a.losses) == 70
    assert torch.equal(a.final_params, b.final_params)
    lines = lambda o: [l for l in o.splitlines() if l.startswith(("[ = =", "loss in worker"))]  # noqa: E731
    assert lines(out_a) == lines(out_b) and len(lines(out_a)) == 140


@pytest.mark.parametrize("comm", ["none", "native"])
def test_minibatch_epoch_graph_same_as_per_step(comm):
    """--batch_size epochs replayed as one graph each (device gathers from a fixed permutation
    buffer, per-step scales baked in, a short last batch) == the per-step loop, bit for bit."""
    kw = dict(device="cuda", widths=[512, 512, 512, 1], n_features=512, n_samples=4000,
              batch_size=1024, lr=1e-5, nepochs=5, comm=comm)
    a = trainer.run_worker(_cfg(**kw))
    b = trainer.run_worker(_cfg(fast_epochs=False, **kw))
    assert a.losses == b.losses and a.steps == b.steps == 20
    assert torch.equal(a.final_params, b.final_params)


def test_compat_cli_wide_preset_takes_the_bench_schedule():
    """``--preset wide8192 --comm native --grad_dtype auto`` through the compat trainer picks what
    bench.py picks: the bf16 payload (auto: > 64 MB of fp32 gradient) and the overlapped chunk
    buckets whose updates ride in the next weight-gradient epilogue (deferred updates).  Without
    ``--grad_dtype`` the CLI keeps the reference's fp32 gradients."""
    from nnmpi_amd.utils.config import build_parser, config_from_args
    assert config_from_args(build_parser().parse_args(["--preset", "wide8192"])).grad_dtype == "fp32"
    cfg = config_from_args(build_parser().parse_args(
        ["--preset", "wide8192", "--comm", "native", "--grad_dtype", "auto", "--nepochs", "2",
         "--print_rank", "none",
         "--data_gen", "device", "--data_dist", "local", "--scaling", "none", "--lr", "1e-5"]))
    res = trainer.run_worker(cfg)
    sch = res.schedule
    assert sch["grad_dtype"] == "bf16" and sch["sync"] == "NativeRcclSync" and not sch["inline"]
    assert sch["deferred_updates"] > 0, sch
    assert all(l == l for l in res.losses)


def test_mpiexec_default_device_on_a_one_gpu_node_matches_golden():
    """`mpiexec -n 2 python dataParallelTraining_NN_MPI.py` with no flags on a node with fewer
    GPUs than ranks: --device auto resolves to the CPU/gloo path (RCCL cannot put two ranks on
    one device) and the reference's P=2 losses come out."""
    import os
    import subprocess
    import sys
    import torch as _t
    if _t.cuda.device_count() >= 2:
        pytest.skip("the node has a GPU per rank")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("MASTER_ADDR", None)
    env.pop("MASTER_PORT", None)
    r = subprocess.run(["/opt/conda/bin/mpiexec", "-n", "2", sys.executable,
                        os.path.join(root, "dataParallelTraining_NN_MPI.py")],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "loss in worker 1: 2835.11" in r.stdout
