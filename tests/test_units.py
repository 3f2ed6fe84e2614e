"""Unit tests (CPU): partitioning, config/CLI typing, dataset, arena layout, bucket plan, ops oracle."""
import numpy as np
import pytest
import torch

import nnmpi_amd
from nnmpi_amd.data.partition import partition_rows
from nnmpi_amd.engine.arena import Arena
from nnmpi_amd.utils.config import TrainConfig, build_parser, config_from_args


@pytest.mark.parametrize("n,p", [(16, 1), (16, 2), (16, 3), (16, 5), (16, 7), (16, 12), (3, 4),
                                 (10_000, 7), (43 * 8, 8)])
def test_partition(n, p):
    part = partition_rows(n, p)
    assert sum(part.counts) == n
    assert part.displs[0] == 0
    for r in range(1, p):
        assert part.displs[r] == part.displs[r - 1] + part.counts[r - 1]
    res = n % p
    for r in range(p):
        assert part.counts[r] == n // p + (1 if r < res else 0)    # reference rule (ref.py:117)


def test_partition_large_counts_no_overflow():
    """Reference D1: int8 element counts overflow above 42 rows/rank."""
    part = partition_rows(1000, 3)
    assert part.element_counts(3) == [1002, 999, 999]


def test_cli_defaults_and_typing():
    a = build_parser().parse_args([])
    cfg = config_from_args(a)
    assert (cfg.lr, cfg.momentum, cfg.batch_size, cfg.nepochs) == (0.001, 0.9, None, 3)
    a = build_parser().parse_args(["--lr", "0.5", "--momentum", "0.1", "--batch_size", "4"])
    cfg = config_from_args(a)
    assert isinstance(cfg.lr, float) and cfg.lr == 0.5 and cfg.batch_size == 4


def test_config_accepts_reference_style_namespace():
    class A:  # the reference's argparse namespace: lr/momentum as strings (D6)
        lr, momentum, batch_size, nepochs = "0.001", "0.9", 4, 3
    cfg = config_from_args(A())
    assert cfg.lr == 0.001 and cfg.batch_size == 4


def test_preset():
    cfg = config_from_args(build_parser().parse_args(["--preset", "mnist"]))
    assert cfg.widths == [784, 1024, 1024, 10] and cfg.loss == "xent"


def test_regression_dataset_numpy_and_tensor():
    X = np.random.RandomState(0).randn(10, 2)
    y = np.arange(10.0)
    ds = nnmpi_amd.RegressionDataset(X, y)
    assert len(ds) == 10 and ds[3][1].item() == 3.0
    assert abs(float(ds.X.mean())) < 1e-12                       # standardized
    ds2 = nnmpi_amd.RegressionDataset(torch.from_numpy(X), torch.from_numpy(y))   # D11 fixed
    assert len(ds2) == 10


def test_arena_layout_and_buckets():
    ar = Arena([(512, 512), (512, 512), (1, 512)], "cpu", bucket_bytes=1 << 20)
    # reverse layer order, 64-element aligned
    assert ar.by_name["layers.4.weight"].offset == 0
    for s in ar.slots:
        assert s.offset % 64 == 0
    covered = sorted((b.offset, b.offset + b.numel) for b in ar.buckets)
    assert covered[0][0] == 0 and covered[-1][1] == ar.numel
    for (s0, e0), (s1, e1) in zip(covered, covered[1:]):
        assert e0 == s1                                          # contiguous, backward order
    assert ar.buckets[0].layers[0] == 2


def test_arena_binds_model_state_dict():
    from nnmpi_amd.models.mlp import reference_init
    m = reference_init()
    ar = Arena([m.spec.layer_shape(i) for i in range(2)], "cpu")
    ar.bind_model(m)
    ar.master.add_(1.0)
    sd = m.state_dict()
    assert torch.equal(sd["layers.0.weight"], ar.weight(0))


def test_torch_ops_match_autograd():
    from nnmpi_amd.ops.torch_ops import TorchOps
    torch.manual_seed(0)
    ops = TorchOps()
    x = torch.randn(32, 8)
    W1, b1 = torch.randn(6, 8, requires_grad=True), torch.randn(6, requires_grad=True)
    W2, b2 = torch.randn(1, 6, requires_grad=True), torch.randn(1, requires_grad=True)
    y = torch.randn(32, 1)
    h = torch.relu(x @ W1.t() + b1)
    out = h @ W2.t() + b2
    loss = torch.nn.functional.mse_loss(out, y)
    loss.backward()
    a = torch.empty(32, 6)
    ops.linear_act(x, W1.detach(), b1.detach(), "relu", a)
    gW2, gb2, dz = torch.empty(1, 6), torch.empty(1), torch.empty(32, 6)
    lo = torch.zeros(4)
    ops.head(a, W2.detach(), b2.detach(), y, None, "mse", 1 / 32, "relu", dz, gW2, gb2,
             torch.empty(32, 1), lo, 1 / 32)
    gW1, gb1 = torch.empty(6, 8), torch.empty(6)
    ops.linear_wgrad(dz, x, gW1, gb1)
    torch.testing.assert_close(lo[0], loss.detach())
    torch.testing.assert_close(gW2, W2.grad)
    torch.testing.assert_close(gb2, b2.grad)
    torch.testing.assert_close(gW1, W1.grad)
    torch.testing.assert_close(gb1, b1.grad)


def test_xent_head_matches_autograd():
    from nnmpi_amd.ops.torch_ops import TorchOps
    torch.manual_seed(1)
    a = torch.relu(torch.randn(16, 12))
    W, b = torch.randn(5, 12, requires_grad=True), torch.randn(5, requires_grad=True)
    lab = torch.randint(0, 5, (16,))
    loss = torch.nn.functional.cross_entropy(a @ W.t() + b, lab)
    loss.backward()
    gW, gb, lo = torch.empty(5, 12), torch.empty(5), torch.zeros(4)
    TorchOps().head(a, W.detach(), b.detach(), None, lab, "xent", 1 / 16, "relu", None, gW, gb,
                    torch.empty(16, 5), lo, 1 / 16)
    torch.testing.assert_close(lo[0], loss.detach())
    torch.testing.assert_close(gW, W.grad)
    torch.testing.assert_close(gb, b.grad)


def test_sgd_variants_match_torch():
    from nnmpi_amd.ops.torch_ops import TorchOps
    for first, nest, wd, damp in [(True, False, 0, 0), (False, True, 0.01, 0), (False, False, 0.01, 0.2)]:
        ar = Arena([(4, 8)], "cpu")
        ar.master.copy_(torch.randn(ar.numel))
        ar.grad.copy_(torch.randn(ar.numel))
        ar.momentum.copy_(torch.randn(ar.numel))
        p = torch.nn.Parameter(ar.master.clone())
        opt = torch.optim.SGD([p], lr=0.1, momentum=0.9, dampening=damp, weight_decay=wd, nesterov=nest)
        if not first:
            opt.state[p]["momentum_buffer"] = ar.momentum.clone()
        p.grad = ar.grad.clone()
        opt.step()
        TorchOps().sgd(ar, torch.tensor([0.1, 0.9, damp, wd, 1.0]), nest, first)
        torch.testing.assert_close(ar.master, p.detach())


def test_chunked_generator_is_partition_independent():
    from nnmpi_amd.data.synth import chunked_regression
    X, y = chunked_regression(0, 3000, 16)
    X2, y2 = chunked_regression(1000, 1500, 16)
    assert torch.equal(X[1000:2500], X2) and torch.equal(y[1000:2500], y2)


def test_engine_cpu_mse_mnist_shapes_run():
    from nnmpi_amd.engine import trainer
    cfg = TrainConfig(device="cpu", print_rank="none", widths=[20, 16, 4], n_features=20, loss="xent",
                      n_samples=64, nepochs=3, lr=0.1)
    res = trainer.run_worker(cfg)
    assert res.losses[-1] < res.losses[0]


def test_watchdog_fires_on_stall():
    import time
    from nnmpi_amd.utils.watchdog import Watchdog
    hit = []
    wd = Watchdog(0.3, None, poll_s=0.05, on_fail=lambda why: hit.append(why))
    time.sleep(0.8)
    wd.stop()
    assert hit and "no training progress" in hit[0]
    # a handler that returns has taken the failure over: the abort backstop must not end the
    # process later (it would kill the rest of the test session with status 3)
    import threading
    assert not [t for t in threading.enumerate() if isinstance(t, threading.Timer) and t.is_alive()]


def test_watchdog_quiet_when_kicked():
    import time
    from nnmpi_amd.utils.watchdog import Watchdog
    hit = []
    wd = Watchdog(0.5, None, poll_s=0.05, on_fail=lambda why: hit.append(why))
    for _ in range(10):
        time.sleep(0.05)
        wd.kick()
    wd.stop()
    assert not hit


def test_sequence_checker_detects_mismatch():
    from nnmpi_amd.utils.seqcheck import CollectiveMismatch, SequenceChecker

    class FakePG:
        def allgather_object(self, obj):
            return [obj, (obj[0], obj[1] + 1)]
    with pytest.raises(CollectiveMismatch):
        SequenceChecker(FakePG()).check(0, 3)


def test_profile_steps_phase_breakdown(capsys):
    from nnmpi_amd.engine import trainer
    cfg = TrainConfig(device="cpu", print_rank="all", widths=[20, 16, 1], n_features=20, n_samples=64,
                      nepochs=3, profile_steps=True)
    res = trainer.run_worker(cfg)
    assert set(res.phase_ms) == {"start->fwd", "fwd->head", "head->bwd", "bwd->comm",
                                 "comm->update"}
    assert all(v >= 0 for v in res.phase_ms.values())
    assert "[profile] mean ms per step" in capsys.readouterr().out


def test_arena_tiny_bucket_merge_and_row_chunks():
    """The few-KB output layer rides with the next layer's bucket; a layer bigger than a bucket
    is cut into output-row chunks (full 256-tile waves), the last chunk holding the bias."""
    ar = Arena([(512, 512), (512, 512), (512, 512), (1, 512)], "meta", bucket_bytes=1 << 20)
    assert [b.layers for b in ar.buckets] == [(3, 2), (1,), (0,)]
    big = Arena([(8192, 8192), (8192, 8192), (1, 8192)], "meta", bucket_bytes=1 << 20)
    assert big.layer_chunks == {0: 4, 1: 4}
    ch = big.chunk_buckets(1)
    assert [b.rows for b in ch] == [(0, 2048), (2048, 4096), (4096, 6144), (6144, 8192)]
    s, e = big.layer_range[1]
    assert ch[0].offset == s and ch[-1].offset + ch[-1].numel == e        # bias in the last
    assert all(b.numel == 2048 * 8192 for b in ch[:-1])
    covered = sorted((b.offset, b.offset + b.numel) for b in big.buckets)
    for (s0, e0), (s1, e1) in zip(covered, covered[1:]):
        assert e0 == s1
    assert big.bucket_of_layer(1) is ch[-1]
    assert big.buckets_completed_by(1) == ch
    # buckets larger than the layer: no chunks
    assert Arena([(8192, 8192), (1, 8192)], "meta", bucket_bytes=1 << 30).layer_chunks == {}


def test_subtract_ranges():
    from nnmpi_amd.parallel.sync import _subtract
    assert _subtract((0, 10), []) == [(0, 10)]
    assert _subtract((0, 10), [(0, 10)]) == []
    assert _subtract((0, 10), [(2, 4), (6, 8)]) == [(0, 2), (4, 6), (8, 10)]
    assert _subtract((5, 10), [(0, 6), (9, 20)]) == [(6, 9)]
    assert _subtract((5, 10), [(10, 12), (0, 5)]) == [(5, 10)]


def test_stale_native_library_is_rebuilt(monkeypatch):
    """A library whose embedded source hash differs from the csrc tree's (sources edited without
    a rebuild) is rebuilt before it is loaded, never run stale."""
    from nnmpi_amd import _build, native
    calls = []
    state = {"built": "0" * 32}
    monkeypatch.setattr(_build, "source_hash", lambda: "f" * 32)
    monkeypatch.setattr(_build, "built_hash", lambda path="": state["built"])

    def fake_build(**kw):
        calls.append(kw)
        state["built"] = "f" * 32
        return _build.ext_path()
    monkeypatch.setattr(_build, "build", fake_build)
    native._load()
    assert len(calls) == 1
    native._load()          # now current: no second build
    assert len(calls) == 1


def test_built_library_carries_the_source_hash():
    from nnmpi_amd import _build
    assert _build.built_hash() == _build.source_hash()


def test_no_mfma_result_read_without_wait_states():
    """Disassemble the built gfx950 code objects and check that no instruction reads an MFMA's
    destination registers without wait states behind the MFMA (the hipcc miss that made the
    general head's one-tile logits kernel store a stale partial sum; nnmpi_amd/_isa_check.py)."""
    import os
    from nnmpi_amd import _build, _isa_check
    if not os.path.exists(_isa_check.OBJDUMP) or not os.path.exists(_build.ext_path()):
        pytest.skip("no llvm-objdump or no built library")
    assert _isa_check.scan_library(_build.ext_path()) == []


def test_rowband_split_host_selection():
    """Which batches the column-split row-band kernel takes (rowband.hip rowband_split_ok, no GPU
    needed): the 512-wide hidden layers, input width 256 / 512, 1-4 hidden layers, up to 128
    bands (4,096 rows) at 2-8 blocks per band, relu / tanh / none; its sync words sit at the
    start of the workspace (the sticky wait-timeout word is int 0), which every batch size
    reserves."""
    from nnmpi_amd import native
    lib = native.lib()
    relu, tanh = 1, 2
    for rows in (1, 37, 1000, 1024, 2048, 3001, 4096):
        assert lib.rowband_split_ok(rows, 512, 512, 3, relu), rows
        assert lib.rowband_split_ok(rows, 512, 512, 3, tanh), rows
    assert lib.rowband_split_ok(999, 512, 256, 1, relu) and lib.rowband_split_ok(999, 512, 512, 4, relu)
    for args in ((4097, 512, 512, 3), (8192, 512, 512, 3), (0, 512, 512, 3), (1024, 256, 256, 3),
                 (1024, 1024, 1024, 2), (1024, 512, 128, 3), (1024, 512, 1024, 3),
                 (1024, 512, 384, 3), (1024, 512, 512, 5)):
        assert not lib.rowband_split_ok(*args, relu), args
    assert lib.rowband_error_word() == 0
    # (the sync area is a fixed prefix: a one-row batch already needs it)
    assert lib.rowband_workspace_bytes(1, 512, 512, 3, 0) >= (32 + 128 * 32) * 4


def test_rowband_host_sizing_invariants():
    """Host-side sizing of the row-band step (rowband.hip), no GPU needed: the engine sizes the
    workspace once for its row capacity and then runs batches of any size up to it, so the bytes
    a batch needs must never exceed the capacity's; the weight-gradient split count is one block
    per CU for the proxy (3 layers x 16 tiles x 5 splits = 240) and >= 4 k-steps per split."""
    from nnmpi_amd import native
    lib = native.lib()
    assert lib.wgrad_multi_splits(3, 512, 512, 8192) == 5
    assert lib.wgrad_multi_splits(1, 512, 512, 8192) == 16
    assert lib.wgrad_multi_splits(3, 512, 512, 512) == 2          # 8 k-steps: >= 4 per split
    assert lib.rowband_blocks(8192) == 256 and lib.rowband_blocks(8191) == 256
    assert lib.rowband_blocks(37) == 2
    cap = lib.rowband_workspace_bytes(8192, 512, 512, 3, 0)
    prev = 0
    for rows in (1, 31, 32, 33, 1000, 4096, 6144, 8000, 8191, 8192):
        need = lib.rowband_workspace_bytes(rows, 512, 512, 3, 0)
        assert prev <= need <= cap, rows
        prev = need
    # a wider input layer needs a larger first-layer slab
    assert lib.rowband_workspace_bytes(8192, 512, 1024, 3, 0) > cap
    assert not lib.rowband2_ok(0, 512, 512, 3, 1, 0, 1)
    # v2 (fragment-major weight images): H in {256, 384, 512, 768, 1024}, input width % 128 == 0,
    # every activation slot + the parameter block in the 160 KiB LDS
    for H, in_, nh in ((512, 512, 3), (512, 512, 4), (256, 256, 4), (384, 128, 2),
                       (768, 768, 3), (1024, 1024, 2), (512, 1024, 2), (256, 512, 1)):
        assert lib.rowband2_ok(8192, H, in_, nh, 1, 0, 1), (H, in_, nh)
        k = [in_] + [H] * (nh - 1)
        assert lib.rowband_packed_elems(H, in_, nh) == sum(H * x for x in k) + H * H * (nh - 1)
    assert not lib.rowband2_ok(8192, 1024, 1024, 3, 1, 0, 1)     # 3 x 64 KiB slots
    assert not lib.rowband2_ok(8192, 512, 784, 3, 1, 0, 1)       # input width % 128
    assert not lib.rowband2_ok(8192, 640, 640, 2, 1, 0, 1)       # H in {256, 384, 512, 768, 1024}
    assert not lib.rowband2_ok(8192, 512, 576, 2, 1, 0, 1)       # in % 128 (ring: k-steps % 2)
    assert not lib.rowband2_ok(8192, 2048, 2048, 1, 1, 0, 1)     # H <= 1024
    assert not lib.rowband2_ok(8192, 512, 512, 3, 10, 1, 1)      # MSE regression head only


def test_rowband_fragment_major_offsets():
    """rb_pk_off (common.h) is a bijection of a [N][K] matrix onto its fragment-major image: 1 KiB
    per 16 x 32 fragment, lane (n & 15) + 16 * ((k >> 3) & 3) holding 8 consecutive k.  Checked
    against the v_mfma_f32_16x16x32_bf16 operand map (cdna_hip_programming.md §3)."""
    N, K = 48, 96
    seen = set()
    for n in range(N):
        for k in range(K):
            frag, rem = divmod(_rb_pk_off(n, k, K), 512)
            lane, e = divmod(rem, 8)
            assert frag == (n // 16) * (K // 32) + k // 32
            assert (lane & 15) == n % 16 and 8 * (lane >> 4) + e == k % 32
            seen.add((frag, lane, e))
    assert len(seen) == N * K


def _rb_pk_off(n, k, K):
    return (((n >> 4) * (K >> 5) + (k >> 5)) * 64 + ((n & 15) + 16 * ((k >> 3) & 3))) * 8 + (k & 7)


def test_shm_allreduce_sums_in_rank_order_and_times_out():
    """The shared-memory all-reduce of CPU ranks (csrc/host/shm_comm.cpp), two handles in one
    process on two threads: every rank gets the rank-ordered fp32 sum (the same bits), repeated
    calls reuse the two slot banks, and a call whose peer never arrives raises instead of hanging."""
    import os
    import secrets
    import threading
    import numpy as np
    from nnmpi_amd import native
    lib = native.lib()
    name = f"/nnmpi-test-{os.getpid()}-{secrets.token_hex(4)}"
    c0 = lib.ShmComm(name, 0, 2, 64, True)
    c1 = lib.ShmComm(name, 1, 2, 64, False)
    c0.unlink()
    rng = np.random.default_rng(0)
    for call in range(5):
        a = rng.standard_normal(37).astype(np.float32)
        b = rng.standard_normal(37).astype(np.float32)
        want = a + b
        bufs = [a.copy(), b.copy()]
        ts = [threading.Thread(target=c.allreduce_sum, args=(buf.ctypes.data, 37, 10.0))
              for c, buf in zip((c0, c1), bufs)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert np.array_equal(bufs[0], want) and np.array_equal(bufs[1], want), call
    lonely = np.ones(8, dtype=np.float32)
    with pytest.raises(RuntimeError, match="stalled"):
        c0.allreduce_sum(lonely.ctypes.data, 8, 0.2)
    with pytest.raises(RuntimeError, match="larger"):
        c1.allreduce_sum(lonely.ctypes.data, 65, 0.2)


def test_shm_sync_matches_gloo_at_two_ranks():
    """Two CPU ranks: the shared-memory all-reduce (default) and gloo give the same parameters bit
    for bit (a + b either way) and the same losses."""
    from _mp import run_ranks_proc
    cfg = dict(device="cpu", print_rank="none", nepochs=5)
    a = run_ranks_proc(cfg, 2)
    b = run_ranks_proc(cfg, 2, env_per_rank=lambda r: {"NNMPI_SHM": "0"})
    assert a[0]["schedule"]["sync"] == "ShmSync" and b[0]["schedule"]["sync"] == "TorchDistSync"
    assert torch.equal(a[0]["final"], a[1]["final"])
    assert torch.equal(a[0]["final"], b[0]["final"])
    assert a[0]["losses"] == b[0]["losses"]


def test_capture_rollback_keeps_the_collective_signature():
    """A graph capture issues no collective: stopping the recording restores the sequence number
    AND the running signature, so a rank that captures one more graph than its peers
    (a partial last mini-batch of its own) still matches them; the failed-capture path too.
    Only the launches (replay) add the recorded notes."""
    from nnmpi_amd.parallel.sync import GradSync
    ar = Arena([(8, 8), (1, 8)], "cpu")
    a, b = GradSync(ar), GradSync(ar)
    for s in (a, b):
        s.note(1, 0, 0, 64, 0)
    # rank a captures an extra graph that holds two collectives, rank b does not
    a.record(True)
    a.note(1, 0, 0, 64, 0)
    a.note(1, 1, 64, 8, 0)
    notes = a.record(False)
    assert len(notes) == 2 and (a.seq, a.sig) == (b.seq, b.sig)
    # a capture that raised: record(False) from the except branch restores the same way
    a.record(True)
    a.note(3, 0, 0, 72, 1)
    a.record(False)
    assert (a.seq, a.sig) == (b.seq, b.sig)
    # one launch of the captured graph on both ranks keeps them equal
    a.replay(notes)
    b.note(1, 0, 0, 64, 0)
    b.note(1, 1, 64, 8, 0)
    assert (a.seq, a.sig) == (b.seq, b.sig)


def test_shm_sync_falls_back_to_gloo_when_one_rank_cannot_load_the_library():
    """the shared-memory all-reduce needs the native library on EVERY rank.  With it
    hidden on rank 1 (NNMPI_NATIVE=0) the ranks agree over gloo and both keep the gloo all-reduce
    (no rank waits in the segment setup); training proceeds and matches the plain-gloo run."""
    from _mp import run_ranks_proc
    cfg = dict(device="cpu", print_rank="none", nepochs=4)
    a = run_ranks_proc(cfg, 2, env_per_rank=lambda r: {"NNMPI_NATIVE": "0"} if r == 1 else {})
    assert a[0]["schedule"]["sync"] == a[1]["schedule"]["sync"] == "TorchDistSync"
    b = run_ranks_proc(cfg, 2, env_per_rank=lambda r: {"NNMPI_SHM": "0"})
    for r in range(2):
        assert a[r]["losses"] == pytest.approx(b[r]["losses"], rel=1e-5)
        assert torch.allclose(a[r]["final"], b[r]["final"], rtol=1e-5, atol=1e-6)


def test_workspace_covers_chunk_bucket_weight_gradients():
    """A layer cut into output-row chunk buckets runs one weight-gradient GEMM per chunk.  A chunk
    has fewer output tiles than the whole layer, so it may split K where the layer does not
    (1024 of 2048 rows at K = 1024: 2 splits, found by the 3-rank wide2048 tuner rehearsal on the
    GPU) -- the engine's split-K workspace must cover the chunk shapes too."""
    from types import SimpleNamespace
    from nnmpi_amd.engine.arena import Arena
    from nnmpi_amd.engine.engine import MLPEngine
    widths = [2048, 2048, 2048, 1]
    arena = Arena([(widths[i + 1], widths[i]) for i in range(3)], "cpu",
                  bucket_bytes=8 * 2 ** 20, chunk_min_tiles=16)
    chunked = [i for i in range(3) if arena.chunk_buckets(i)]
    assert chunked, "the 2048-wide layers must be cut into chunk buckets"

    class Ops:   # a chunk splits, the whole layer does not
        def wgrad_workspace_bytes(self, rows, out_f, in_f, dtype):
            return 0 if out_f == 2048 else 1000 + out_f

        def head_workspace_bytes(self, rows, in_f, out_f):
            return 0

    stub = SimpleNamespace(ops=Ops(), R=1024, spec=SimpleNamespace(widths=widths), L=3,
                           arena=arena, dtype=torch.bfloat16, use_tiny=False)
    rows = max(b.rows[1] - b.rows[0] for i in chunked for b in arena.chunk_buckets(i))
    assert MLPEngine._workspace_bytes(stub) == 1000 + rows


def _xcd_remap(bid, nwg):
    """Host replica of csrc/kernels/common.h xcd_remap (block id -> work id)."""
    if nwg <= 8:
        return bid
    q, r, xcd = nwg // 8, nwg % 8, bid % 8
    return (xcd * (q + 1) if xcd < r else r * (q + 1) + (xcd - r) * q) + bid // 8


@pytest.mark.parametrize("nwg", [1, 7, 8, 9, 31, 256, 257, 300, 1023, 1024])
def test_xcd_remap_is_a_permutation_with_contiguous_xcd_ranges(nwg):
    """The row-band kernel's XCD-contiguous band order (RowbandArgs::band_map) and the grouped
    weight gradients use xcd_remap: every band must be run exactly once, and the blocks that
    share an XCD (same id mod 8) must get one contiguous range of work ids."""
    ids = [_xcd_remap(b, nwg) for b in range(nwg)]
    assert sorted(ids) == list(range(nwg))
    if nwg > 8:
        for x in range(8):
            mine = sorted(ids[b] for b in range(x, nwg, 8))
            assert mine == list(range(mine[0], mine[0] + len(mine)))


def test_knob_without_experiments_switch_is_ignored_and_reported():
    """Production gating (conftest turns NNMPI_EXPERIMENTS on for the suite, so this runs in a
    clean subprocess): without NNMPI_EXPERIMENTS=1 a knob keeps its default, and the trainer's
    check names it on stderr."""
    import os
    import subprocess
    import sys
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if not k.startswith("NNMPI_")}
    env["NNMPI_ROWBAND"] = "0"
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from nnmpi_amd.utils import knobs\n"
            "from nnmpi_amd.engine.trainer import _warn_ignored_knobs\n"
            "assert knobs.knob('NNMPI_ROWBAND', '1') == '1'\n"
            "assert _warn_ignored_knobs(0) == ['NNMPI_ROWBAND']\n") % ROOT
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "NNMPI_ROWBAND set but not honoured" in r.stderr
