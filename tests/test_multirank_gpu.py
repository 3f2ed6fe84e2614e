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
from test_golden import GOLDEN_LOSSES, GOLDEN_PARAMS

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


def test_rccl_grouped_overlap_two_ranks_bitwise():
    """512-wide (grouped backward kernels) at P=2: per-bucket all-reduce overlapped on the comm
    stream == one inline all-reduce == the gloo all-reduce, bit for bit."""
    kw = dict(widths=[512, 512, 512, 1], n_features=512, n_samples=4096, lr=1e-4)
    a = run_ranks_proc(_cfg(comm="native", comm_mode="overlap", **kw), 2, env_per_rank=rccl_env)
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
