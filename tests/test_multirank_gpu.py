"""The GPU engine at P >= 2 -- several rank processes sharing one MI355X.

Two transports make that possible on a one-GPU box:

* ``comm="gloo"``: the gradient all-reduce of device tensors over gloo (TorchDistSync) while
  every kernel is the HIP path (HipOps) -- the reference semantics at P = 2/3/4 on the GPU
  kernels: the 1/P gradient scale, uneven and empty shards, per-rank graph keys.
* ``comm="native"``: the C++ RCCL runtime itself.  RCCL refuses two ranks on one device
  ("Duplicate GPU detected") unless they look like different hosts: each rank gets its own
  ``NCCL_HOSTID``, so the ranks meet over RCCL's network transport on the loopback interface.
  Slow, but it is the real data plane: ncclAllReduce / ReduceScatter / AllGather / Broadcast /
  grouped Send-Recv, captured in the step's hipGraph, with P > 1.

Reference: the gather -> root average -> send pattern these replace (ref.py:185-211).
"""
import pytest
import torch

from _mp import run_ranks_proc
from test_golden import GOLDEN_LOSSES, GOLDEN_P12, GOLDEN_P12_PARAMS, GOLDEN_PARAMS

pytestmark = pytest.mark.gpu


def rccl_env(rank):
    return {"NCCL_HOSTID": f"nnmpi-test-host-{rank}", "NCCL_SOCKET_IFNAME": "lo",
            "NCCL_IB_DISABLE": "1", "PYTHONFAULTHANDLER": "1", "NCCL_DEBUG": "WARN"}


def _cfg(**kw):
    base = dict(device="cuda", print_rank="none", widths=[256, 256, 256, 1], n_features=256,
                n_samples=2048, dtype="bf16", nepochs=4, lr=1e-3, data_gen="device",
                data_dist="local", scaling="none")
    base.update(kw)
    return base


def _replicas_equal(out):
    for r in range(1, len(out)):
        assert torch.equal(out[r]["final"], out[0]["final"]), f"rank {r} diverged"


# ---------------------------------------------------------------- gloo transport, HIP kernels
@pytest.mark.parametrize("world", [2, 4])
def test_reference_golden_on_gpu_kernels(world):
    """SURVEY §4.2 goldens at P=2/4 through the tiny-MLP kernel (per-shard scaling,
    unweighted average, rank-0 scatter)."""
    out = run_ranks_proc(dict(device="cuda", comm="gloo", print_rank="none", graph=False), world)
    for r in range(world):
        assert out[r]["losses"] == pytest.approx(GOLDEN_LOSSES[world][r], rel=1e-5), r
        assert torch.allclose(out[r]["final"], torch.tensor(GOLDEN_PARAMS[world]), atol=5e-6)
    _replicas_equal(out)


def test_bf16_512_global_weighted_p2_matches_p1():
    """Global feature scaling + weighted averaging: P=2 computes the P=1 gradient (up to the
    fp32 summation split and the bf16 rounding that follows it)."""
    kw = dict(widths=[512, 512, 512, 1], n_features=512, n_samples=4096, scaling="global",
              averaging="weighted", lr=1e-4, nepochs=4, graph=False)
    one = run_ranks_proc(_cfg(comm="none", **kw), 1)
    two = run_ranks_proc(_cfg(comm="gloo", **kw), 2)
    _replicas_equal(two)
    torch.testing.assert_close(two[0]["final"], one[0]["final"], rtol=2e-2, atol=2e-3)
    g1 = one[0]["losses"]
    g2 = [(a * 2048 + b * 2048) / 4096 for a, b in zip(two[0]["losses"], two[1]["losses"])]
    assert g2 == pytest.approx(g1, rel=1e-2)


def test_uneven_three_ranks_and_empty_shard():
    """Uneven split (334/334/333 rows) and an EMPTY shard (2 rows over 3 ranks) on the
    default (overlapped) schedule: every rank joins every collective, replicas stay bitwise
    equal."""
    out = run_ranks_proc(_cfg(comm="gloo", n_samples=1001, graph=False), 3)
    assert [o["rows"] for o in out] == [334, 334, 333]
    _replicas_equal(out)
    out = run_ranks_proc(_cfg(comm="gloo", n_samples=2, graph=False), 3)
    assert [o["rows"] for o in out] == [1, 1, 0]
    _replicas_equal(out)
    assert all(l == l for l in out[0]["losses"])


def test_short_shard_empty_minibatches():
    """--batch_size with a short shard: the last micro-batch of rank 2 is empty."""
    out = run_ranks_proc(_cfg(comm="gloo", n_samples=600, batch_size=128, nepochs=2,
                              graph=False), 3)
    assert all(o["steps"] == out[0]["steps"] for o in out)
    _replicas_equal(out)


def test_zero1_gloo_bitwise_equal_allreduce():
    a = run_ranks_proc(_cfg(comm="gloo", shard_optimizer=True, graph=False), 2)
    b = run_ranks_proc(_cfg(comm="gloo", graph=False), 2)
    _replicas_equal(a)
    assert torch.equal(a[0]["final"], b[0]["final"])
    assert a[0]["losses"] == b[0]["losses"]


# ---------------------------------------------------------------- the RCCL runtime, P = 2 / 3
def test_rccl_two_ranks_bitwise_equal_gloo():
    """Two-rank ncclAllReduce (inline, captured in the step graph) == the gloo all-reduce of
    the same gradients: a + b is the same fp32 sum either way."""
    a = run_ranks_proc(_cfg(comm="native"), 2, env_per_rank=rccl_env)
    b = run_ranks_proc(_cfg(comm="gloo", graph=False), 2)
    _replicas_equal(a)
    assert a[0]["losses"] == b[0]["losses"] and a[1]["losses"] == b[1]["losses"]
    assert torch.equal(a[0]["final"], b[0]["final"])


@pytest.mark.parametrize("graph", [False, True])
def test_rccl_overlap_two_ranks_runs(graph):
    out = run_ranks_proc(_cfg(comm="native", comm_mode="overlap", graph=graph, nepochs=2), 2,
                         env_per_rank=rccl_env)
    _replicas_equal(out)


@pytest.mark.parametrize("mode", ["overlap", "inline"])
def test_rccl_schedules_bitwise_equal(mode):
    """Per-bucket all-reduce on the comm stream (small buckets) and the inline form give the
    same parameters bit for bit at P=2, as does the eager (no graph) run."""
    kw = dict(comm="native", comm_mode=mode, bucket_mb=0.05)
    a = run_ranks_proc(_cfg(**kw), 2, env_per_rank=rccl_env)
    b = run_ranks_proc(_cfg(graph=False, **kw), 2, env_per_rank=rccl_env)
    c = run_ranks_proc(_cfg(comm="gloo", graph=False), 2)
    _replicas_equal(a)
    assert torch.equal(a[0]["final"], b[0]["final"])
    assert torch.equal(a[0]["final"], c[0]["final"])


def test_rccl_zero1_bf16_shadow_replicas_equal():
    """ZeRO-1 over RCCL with a bf16 shadow: reduce-scatter, owner SGD, bf16 all-gather plus the
    fp32 refresh of the head and bias pieces -- every rank keeps computing with the same
    parameters, equal to the all-reduce run."""
    a = run_ranks_proc(_cfg(comm="native", shard_optimizer=True), 2, env_per_rank=rccl_env)
    b = run_ranks_proc(_cfg(comm="native"), 2, env_per_rank=rccl_env)
    _replicas_equal(a)
    assert a[0]["losses"] == b[0]["losses"] and a[1]["losses"] == b[1]["losses"]
    assert torch.equal(a[0]["final"], b[0]["final"])


def test_rccl_bf16_payload_three_ranks_uneven_and_empty():
    out = run_ranks_proc(_cfg(comm="native", grad_dtype="bf16", comm_mode="overlap",
                              n_samples=1001), 3, env_per_rank=rccl_env)
    _replicas_equal(out)
    out = run_ranks_proc(_cfg(comm="native", n_samples=2), 3, env_per_rank=rccl_env)
    assert [o["rows"] for o in out] == [1, 1, 0]
    _replicas_equal(out)


def test_rccl_reference_golden_p2_scatterv():
    """Reference config over RCCL: rank-0 data + grouped ncclSend/Recv scatter, broadcast of
    the initial model, tiny kernel, all-reduce: the P=2 goldens."""
    out = run_ranks_proc(dict(device="cuda", comm="native", print_rank="none"), 2,
                         env_per_rank=rccl_env)
    for r in range(2):
        assert out[r]["losses"] == pytest.approx(GOLDEN_LOSSES[2][r], rel=1e-5), r
        assert torch.allclose(out[r]["final"], torch.tensor(GOLDEN_PARAMS[2]), atol=5e-6)
    _replicas_equal(out)


@pytest.mark.parametrize("world", [3, 12])
def test_rccl_reference_uneven_scatterv_matches_cpu(world):
    """The reference config with an UNEVEN split over RCCL (BASELINE config 3's "uneven dataset
    split"): rank 0 generates the 16 rows and scatters them with grouped ncclSend/Recv of
    per-rank counts (the reference's Bcast(counts) + Scatterv, ref.py:110-143; it crashes at P=3,
    D2), the model is broadcast, the tiny kernel steps, the gradient is all-reduced.  Every rank
    matches the CPU (gloo) run of the same job to rtol 1e-5, replicas are bitwise equal, and at
    P = 12 ranks 0 and 11 match the reference's own output."""
    cfg = dict(print_rank="none", data_dist="scatter")
    gpu = run_ranks_proc(dict(cfg, device="cuda", comm="native"), world, env_per_rank=rccl_env,
                         timeout=420.0)
    cpu = run_ranks_proc(dict(cfg, device="cpu"), world, timeout=300.0)
    rows = [o["rows"] for o in gpu]
    assert sum(rows) == 16 and rows == [o["rows"] for o in cpu] and len(set(rows)) == 2
    for r in range(world):
        assert gpu[r]["losses"] == pytest.approx(cpu[r]["losses"], rel=1e-5), r
        assert torch.allclose(gpu[r]["final"], cpu[r]["final"], rtol=1e-5, atol=1e-6), r
    _replicas_equal(gpu)
    if world == 12:
        for r, want in GOLDEN_P12.items():
            assert gpu[r]["losses"] == pytest.approx(want, rel=1e-5), r
        assert torch.allclose(gpu[0]["final"], torch.tensor(GOLDEN_P12_PARAMS), atol=5e-6)


def test_rccl_grouped_overlap_two_ranks_bitwise():
    """512-wide (grouped backward kernels) at P=2: per-bucket all-reduce overlapped on the comm
    stream == one inline all-reduce == the gloo all-reduce, bit for bit."""
    kw = dict(widths=[512, 512, 512, 1], n_features=512, n_samples=4096, lr=1e-4)
    # (--seqcheck: the per-epoch collective signature, replayed graphs included, agrees)
    a = run_ranks_proc(_cfg(comm="native", comm_mode="overlap", seqcheck=True, **kw), 2,
                       env_per_rank=rccl_env)
    b = run_ranks_proc(_cfg(comm="native", comm_mode="inline", **kw), 2, env_per_rank=rccl_env)
    c = run_ranks_proc(_cfg(comm="gloo", graph=False, **kw), 2)
    _replicas_equal(a)
    assert torch.equal(a[0]["final"], b[0]["final"])
    assert torch.equal(a[0]["final"], c[0]["final"])


@pytest.mark.parametrize("grad_dtype", ["fp32", "bf16"])
def test_rccl_chunked_buckets_two_ranks_bitwise(grad_dtype):
    """Sub-layer (output-row chunk) buckets at P=2 on 1024-wide layers (chunking forced small
    with NNMPI_CHUNK_MIN_TILES): chunk all-reduces overlapped == inline, bit for bit.  With the
    bf16 payload (256 rows per rank: un-split weight gradients) the overlapped chunks' GEMM
    epilogues write the bf16 payload themselves."""
    kw = dict(widths=[1024, 1024, 1024, 1], n_features=1024, lr=1e-4, bucket_mb=1.0,
              grad_dtype=grad_dtype, n_samples=1024 if grad_dtype == "fp32" else 512)

    def env(r):
        return dict(rccl_env(r), NNMPI_CHUNK_MIN_TILES="4")
    a = run_ranks_proc(_cfg(comm="native", comm_mode="overlap", **kw), 2, env_per_rank=env)
    b = run_ranks_proc(_cfg(comm="native", comm_mode="inline", **kw), 2, env_per_rank=env)
    _replicas_equal(a)
    assert torch.equal(a[0]["final"], b[0]["final"])


# ---------------------------------------------------------------- bf16 payload numerics, P > 2
def _bf16_reduce_job(world, n=300_007):
    return run_ranks_proc({"n": n}, world, env_per_rank=rccl_env, timeout=240,
                          entry="_rccl_reduce_entry.py")


def _rel(x, exact):
    return float((x.double() - exact).norm() / exact.norm())


@pytest.mark.parametrize("world", [3, 4, 8])
def test_rccl_bf16_reduction_error_vs_p(world):
    """The bf16 gradient payload's reduction at P = 3 / 4 / 8 (ranks sharing the GPU).

    * acc32 (the default): bitwise equal on every rank to bf16(sum over ranks, in rank order, in
      fp32, of bf16(g_r)) -- one rounding of the inputs, one of the sum, whatever P is -- so its
      error against the exact sum of the fp32 gradients stays at the bf16 half-ulp level
      (<= 2^-8 relative per element).
    * ncclAllReduce in bf16 is measured next to it (its ring rounds the partial sum at every
      hop) and both errors are written to gpurun_out/ for the record; only acc32 is pinned.
    The reference averages fp32 gradients exactly (ref.py:190-197)."""
    out = _bf16_reduce_job(world)
    g = [o["g"] for o in out]
    exact = torch.stack([x.double() for x in g]).sum(0)
    emul = torch.zeros_like(g[0])
    for x in g:                                  # fp32 accumulation in rank order
        emul += x.to(torch.bfloat16).float()
    emul = emul.to(torch.bfloat16)
    for r, o in enumerate(out):
        assert torch.equal(o["acc32"], emul), f"rank {r}: acc32 differs from its contract"
        assert torch.equal(o["acc32"], out[0]["acc32"]) and torch.equal(o["ring_bf16"], out[0]["ring_bf16"])
    e_acc, e_ring = _rel(out[0]["acc32"], exact), _rel(out[0]["ring_bf16"], exact)
    e_f32 = _rel(out[0]["fp32"], exact)
    # elementwise: every bf16 rounding (8 significant bits) is within u = 2^-8 relative: the
    # inputs' roundings add up to u * sum|g_r|, the output's to u * |sum| (+ second order)
    u = 2.0 ** -8
    bound = (torch.stack([x.double().abs() for x in g]).sum(0) * u * (1 + 2 * u) +
             exact.abs() * u * (1 + 2 * u) + 1e-30)
    assert bool(((out[0]["acc32"].double() - exact).abs() <= bound).all())
    assert e_acc < 8e-3 and e_f32 < 1e-6
    import json
    import os
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/bf16_reduce_error.jsonl", "a") as f:
        f.write(json.dumps({"world": world, "n": int(exact.numel()), "rel_err_acc32": e_acc,
                            "rel_err_rccl_bf16_ring": e_ring, "rel_err_fp32": e_f32}) + "\n")


@pytest.mark.parametrize("world", [3, 4])
def test_rccl_bf16_payload_training_close_to_fp32(world):
    """~20 steps of a 1024x3 model with chunk buckets forced, bf16 payload (acc32 reduction,
    overlapped chunk all-reduces, deferred updates) vs the fp32 payload at P = 3 / 4:
    replicas bitwise equal, and the parameter UPDATE within 1e-2 relative (L2) of the fp32
    run's.  Justification: each step's reduced gradient differs from the fp32 one by at most
    the two bf16 roundings (2^-9 relative each per element, ~0.4 % worst case, ~0.2 % typical);
    the update is a momentum average of such gradients times lr, so its relative error stays
    at that level over 20 small steps -- 1e-2 leaves a 2.5x margin over the worst case."""
    kw = dict(widths=[1024, 1024, 1024, 1], n_features=1024, lr=1e-4, bucket_mb=1.0,
              n_samples=256 * world, nepochs=20, comm_mode="overlap")

    def env(r):
        return dict(rccl_env(r), NNMPI_CHUNK_MIN_TILES="4")
    init = run_ranks_proc(_cfg(comm="none", nepochs=0, **{k: v for k, v in kw.items()
                                                          if k != "nepochs"}), 1)[0]["final"]
    b16 = run_ranks_proc(_cfg(comm="native", grad_dtype="bf16", **kw), world, env_per_rank=env,
                         timeout=300)
    f32 = run_ranks_proc(_cfg(comm="native", grad_dtype="fp32", **kw), world, env_per_rank=env,
                         timeout=300)
    _replicas_equal(b16)
    _replicas_equal(f32)
    du16, du32 = b16[0]["final"] - init, f32[0]["final"] - init
    assert float(du32.norm()) > 0
    rel = float((du16 - du32).norm() / du32.norm())
    assert rel < 1e-2, rel


# ---------------------------------------------------------------- failure path over RCCL
def test_rccl_one_rank_failure_ends_every_rank():
    """The GPU twin of test_parallel_cpu.py::test_one_rank_failure_ends_every_rank: 3 RCCL ranks
    (graph-replayed steps, the all-reduce captured in the step's hipGraph), rank 1 raising at
    epoch 1 while ranks 0 and 2 wait inside the captured collective.  The reference hangs here
    (ref.py:185,203).  Every rank must exit non-zero within timeout_s + 30 s
    (after start-up), the survivors through the watchdog, which aborts the communicator
    (ncclCommAbort) so the spinning collective kernels return."""
    import os
    import subprocess
    import sys
    import time
    from _mp import _free_port
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    timeout_s, world, fail = 20, 3, 1
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   NNMPI_FAULT_INJECT=f"{fail}:1", OMP_NUM_THREADS="1", **rccl_env(r))
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(root, "dataParallelTraining_NN_MPI.py"), "--device",
             "cuda", "--comm", "native", "--nepochs", "40", "--timeout_s", str(timeout_s),
             "--print_rank", "none"], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
            text=True))
    t_fail = None
    deadline = time.monotonic() + 240
    try:
        while any(p.poll() is None for p in procs) and time.monotonic() < deadline:
            if t_fail is None and procs[fail].poll() is not None:
                t_fail = time.monotonic()
            time.sleep(0.2)
        t_end = time.monotonic()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    errs = [p.stderr.read() for p in procs]
    codes = [p.returncode for p in procs]
    assert all(c not in (None, 0) for c in codes), (codes, [e[-2000:] for e in errs])
    assert "injected fault" in errs[fail]
    assert t_fail is not None and t_end - t_fail < timeout_s + 30, (t_end - t_fail, codes)
    for r in range(world):
        if r != fail:
            assert "nnmpi watchdog" in errs[r] or "RCCL" in errs[r], errs[r][-2000:]


@pytest.mark.rowband
def test_rowband_rccl_two_ranks_inline_and_zero1_match_one_rank():
    """The row-band step at P=2 through RCCL (inline all-reduce, and ZeRO-1's reduce-scatter /
    sharded update / all-gather): replicas bitwise equal, the two syncs bitwise equal to each
    other (a + b either way), and the P=1 trajectory of the same global data within the bf16
    contract (the split of the batch changes the fp32 summation order of the weight gradients)."""
    kw = dict(widths=[512, 512, 512, 1], n_features=512, n_samples=4096, scaling="global",
              averaging="weighted", lr=1e-4, nepochs=4)
    one = run_ranks_proc(_cfg(comm="none", **kw), 1)
    a = run_ranks_proc(_cfg(comm="native", comm_mode="inline", **kw), 2, env_per_rank=rccl_env)
    b = run_ranks_proc(_cfg(comm="native", comm_mode="inline", shard_optimizer=True, **kw), 2,
                       env_per_rank=rccl_env)
    assert one[0]["schedule"]["rowband"] and a[0]["schedule"]["rowband"] and b[0]["schedule"]["rowband"]
    _replicas_equal(a)
    _replicas_equal(b)
    assert torch.equal(a[0]["final"], b[0]["final"])
    torch.testing.assert_close(a[0]["final"], one[0]["final"], rtol=2e-2, atol=2e-3)



@pytest.mark.rowband
@pytest.mark.parametrize("world", [2, 3])
def test_rowband_overlap_matches_inline_bitwise(world):
    """The overlapped row-band schedule (--comm_mode overlap_rowband: the last hidden layer's and
    the head's bucket all-reduced on the comm stream while the other layers' weight gradients
    compute, each bucket's SGD -- which also refreshes its layers' v2 images -- behind its
    collective) against the inline row-band sync with the same split-K plan
    (NNMPI_RB_PLAN=1): RCCL ranks sharing the GPU, an uneven split at P=3, bitwise-equal
    parameters and losses, replicas bitwise equal."""
    kw = dict(widths=[512, 512, 512, 512, 1], n_features=512, n_samples=2048 * world - 1,
              lr=1e-4, nepochs=4)
    # one fp32 reduction for both: the inline schedule's single bucket defaults to ncclAllReduce
    a = run_ranks_proc(_cfg(comm="native", comm_mode="overlap_rowband", **kw), world,
                       env_per_rank=lambda r: dict(rccl_env(r), NNMPI_F32_REDUCE="ordered"),
                       timeout=300.0)
    b = run_ranks_proc(_cfg(comm="native", comm_mode="inline", **kw), world,
                       env_per_rank=lambda r: dict(rccl_env(r), NNMPI_RB_PLAN="1",
                                                   NNMPI_F32_REDUCE="ordered"), timeout=300.0)
    for o in a + b:
        assert o["schedule"]["rowband"], o["schedule"]
    _replicas_equal(a)
    _replicas_equal(b)
    assert torch.equal(a[0]["final"], b[0]["final"])
    for r in range(world):
        assert a[r]["losses"] == b[r]["losses"], r
