"""Multi-rank behaviour on CPU (gloo): uneven splits, DP == single-process equivalence, sync
modes, mini-batches, sequence checker, checkpoint/resume, launchers."""
import os
import shutil
import subprocess
import sys

import pytest
import torch

from _mp import _free_port, run_ranks

import nnmpi_amd  # noqa: F401
from nnmpi_amd.engine import trainer
from nnmpi_amd.utils.config import TrainConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [3, 5, 6, 7])
def test_uneven_world_sizes_train(world):
    """The reference crashes for P in {3,5,6,7} (int8 counts as MPI.INT, D2); here they train."""
    out = run_ranks(TrainConfig(device="cpu", print_rank="none"), world)
    rows = [o["rows"] for o in out]
    assert sum(rows) == 16 and max(rows) - min(rows) <= 1
    for o in out:
        assert torch.equal(o["final"], out[0]["final"])           # replicas identical
        assert all(l == l for l in o["losses"])                    # finite


def test_more_ranks_than_rows_allows_empty_shards():
    cfg = TrainConfig(device="cpu", print_rank="none", n_samples=3, averaging="weighted", scaling="global")
    out = run_ranks(cfg, 4)
    assert [o["rows"] for o in out] == [1, 1, 1, 0]
    for o in out:
        assert torch.equal(o["final"], out[0]["final"])


@pytest.mark.parametrize("world", [2, 3, 4])
def test_dp_equals_single_process_with_global_scaling(world):
    """With global feature scaling and sample-weighted averaging, P-rank DP == 1 rank."""
    cfg = TrainConfig(device="cpu", print_rank="none", scaling="global", averaging="weighted", nepochs=6,
                      n_samples=48, lr=0.01)
    single = trainer.run_worker(cfg)
    out = run_ranks(cfg, world)
    for o in out:
        torch.testing.assert_close(o["final"], single.final_params, rtol=1e-5, atol=2e-6)


def test_root_sync_mode_matches_allreduce():
    a = run_ranks(TrainConfig(device="cpu", print_rank="none", sync="root"), 4)
    b = run_ranks(TrainConfig(device="cpu", print_rank="none", sync="allreduce"), 4)
    for x, y in zip(a, b):
        torch.testing.assert_close(x["final"], y["final"], rtol=1e-5, atol=2e-6)


def test_minibatches_uneven_ranks_do_not_deadlock():
    cfg = TrainConfig(device="cpu", print_rank="none", batch_size=2, n_samples=17, nepochs=2)
    out = run_ranks(cfg, 3)
    for o in out:
        assert o["steps"] == 2 * 3          # ceil(6 rows / 2) steps per epoch on every rank
        assert torch.equal(o["final"], out[0]["final"])


def test_sequence_checker_passes():
    out = run_ranks(TrainConfig(device="cpu", print_rank="none", seqcheck=True), 2)
    assert len(out) == 2


def test_sequence_checker_catches_bucket_layout_mismatch():
    """Two ranks with different bucket layouts (rank 1 chunks the 512x512 layer into row
    buckets, rank 0 does not) issue the same number of collectives with different sizes -- a
    hang or silent corruption over RCCL.  --seqcheck compares the plans before the first
    collective and every rank raises instead."""
    from _mp import run_ranks_proc
    cfg = dict(device="cpu", print_rank="none", widths=[512, 512, 1], n_features=512,
               n_samples=64, bucket_mb=0.1, seqcheck=True, nepochs=2, data_gen="device",
               data_dist="local")
    # (per-bucket gloo collectives: the shared-memory sync reduces one whole-arena bucket)
    with pytest.raises(AssertionError, match="CollectiveMismatch"):
        run_ranks_proc(cfg, 2, env_per_rank=lambda r: ({"NNMPI_CHUNK_MIN_TILES": "1", "NNMPI_SHM": "0"}
                                                      if r else {"NNMPI_SHM": "0"}))
    out = run_ranks_proc(cfg, 2, env_per_rank=lambda r: {"NNMPI_SHM": "0"})   # same layout: passes
    assert torch.equal(out[0]["final"], out[1]["final"])


def test_bf16_cpu_path_trains():
    cfg = TrainConfig(device="cpu", print_rank="none", widths=[64, 64, 64, 1], n_features=64, n_samples=512,
                      dtype="bf16", nepochs=4, lr=1e-4)
    out = run_ranks(cfg, 2)
    assert out[0]["losses"][-1] < out[0]["losses"][0]
    assert torch.equal(out[0]["final"], out[1]["final"])


def test_checkpoint_resume_is_exact(tmp_path):
    ck = str(tmp_path / "model.pt")
    full = trainer.run_worker(TrainConfig(device="cpu", print_rank="none", nepochs=5))
    trainer.run_worker(TrainConfig(device="cpu", print_rank="none", nepochs=3, checkpoint=ck))
    res = trainer.run_worker(TrainConfig(device="cpu", print_rank="none", nepochs=5, resume=ck))
    assert torch.equal(res.final_params, full.final_params)
    sd = torch.load(ck, weights_only=True)
    assert list(sd) == ["layers.0.weight", "layers.0.bias", "layers.2.weight", "layers.2.bias"]
    # the saved state_dict loads into the reference-shaped module
    from nnmpi_amd.models.mlp import MLP
    MLP().load_state_dict(sd)


def test_metrics_json(tmp_path):
    mj = str(tmp_path / "m.jsonl")
    trainer.run_worker(TrainConfig(device="cpu", print_rank="none", metrics_json=mj))
    import json
    lines = [json.loads(l) for l in open(mj)]
    assert len(lines) == 3 and all("samples_per_s" in l for l in lines)


def test_metrics_comm_volume_and_efficiency(tmp_path):
    """per-rank wire bytes of the gradient sync and S(P)/(P*S(1))."""
    import json
    from nnmpi_amd.utils.metrics import comm_bus_gbps, comm_volume, parallel_efficiency
    v = comm_volume(1000, 4)
    assert v == {"grad_bytes": 4000, "wire_bytes_per_rank": 6000}       # 2*(3/4)*4000
    z = comm_volume(1000, 4, sharded=True, shadow=True)
    assert z["wire_bytes_per_rank"] == 3000 + 1500                         # RS fp32 + AG bf16
    assert comm_volume(1000, 1)["wire_bytes_per_rank"] == 0
    assert abs(comm_bus_gbps(6000, 0.001) - 6.0) < 1e-9
    assert parallel_efficiency(300.0, 4, 100.0) == 0.75
    assert parallel_efficiency(300.0, 4, None) is None
    mj = str(tmp_path / "m.jsonl")
    run_ranks(TrainConfig(device="cpu", print_rank="none", metrics_json=mj, ref_samples_per_s=1000.0), 2)
    lines = [json.loads(l) for l in open(mj)]
    assert lines and all(l["world"] == 2 for l in lines)
    # 13 parameters padded into the 64-aligned arena, fp32 ring all-reduce over 2 ranks
    assert all(l["wire_bytes_per_rank"] == l["grad_bytes"] for l in lines)
    assert all(abs(l["parallel_efficiency"] - l["samples_per_s"] / 2000.0) < 1e-9 for l in lines)


def test_cli_single_process_prints_reference_lines():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "dataParallelTraining_NN_MPI.py")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert lines[0] == "[ = = = = = Epoch 0 = = = = = ]"
    assert lines[1].startswith("loss in worker 0: 2530.83")
    assert len(lines) == 6


def test_cli_typed_flags():
    """Reference D6: --lr/--momentum overrides must be floats (the reference crashes)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "dataParallelTraining_NN_MPI.py"),
                        "--lr", "0.002", "--momentum", "0.5", "--nepochs", "1"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "loss in worker 0:" in r.stdout


@pytest.mark.skipif(not os.path.exists("/opt/conda/bin/mpiexec"), reason="no mpiexec")
def test_mpiexec_launch_matches_golden():
    """`mpiexec -n 2 python dataParallelTraining_NN_MPI.py` (README.md:12) via PMI env."""
    env = dict(os.environ)
    env.pop("MASTER_ADDR", None)
    env.pop("MASTER_PORT", None)
    r = subprocess.run(["/opt/conda/bin/mpiexec", "-n", "2", sys.executable,
                        os.path.join(ROOT, "dataParallelTraining_NN_MPI.py"), "--device", "cpu"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    got = {}
    for l in r.stdout.splitlines():
        if l.startswith("loss in worker"):
            rk = int(l.split()[3].rstrip(":"))
            got.setdefault(rk, []).append(float(l.split()[-1]))
    assert got[0] == pytest.approx([2230.0779, 2227.2249, 2221.5249], rel=1e-5)
    assert got[1] == pytest.approx([2835.1191, 2831.0088, 2822.7886], rel=1e-5)


def test_self_spawn_cli():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "dataParallelTraining_NN_MPI.py"),
                        "--nprocs", "2", "--nepochs", "1", "--device", "cpu"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "loss in worker 1: 2835.11" in r.stdout


def test_bf16_gradient_payload_trains_close_to_fp32():
    """--grad_dtype bf16: the all-reduce payload is rounded to bf16 (half the xGMI bytes);
    replicas stay identical and the run tracks the fp32-payload run closely."""
    cfg = dict(print_rank="none", n_samples=64, nepochs=5, lr=0.01)
    a = run_ranks(TrainConfig(device="cpu", grad_dtype="bf16", **cfg), 2)
    b = run_ranks(TrainConfig(device="cpu", grad_dtype="fp32", **cfg), 2)
    assert torch.equal(a[0]["final"], a[1]["final"])
    torch.testing.assert_close(a[0]["final"], b[0]["final"], rtol=2e-2, atol=2e-3)
    assert not torch.equal(a[0]["final"], b[0]["final"])   # the rounding really happened


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_optimizer_matches_allreduce_bitwise(world):
    """ZeRO-1 (reduce-scatter -> SGD on the own 1/P slice -> all-gather) computes exactly the
    all-reduce path's update; world 3 leaves an uneven data split and a padded arena."""
    cfg = dict(print_rank="none", nepochs=4, n_samples=17)
    a = run_ranks(TrainConfig(device="cpu", shard_optimizer=True, **cfg), world)
    b = run_ranks(TrainConfig(device="cpu", **cfg), world)
    for x, y in zip(a, b):
        assert x["losses"] == y["losses"]
        assert torch.equal(x["final"], y["final"])


def test_sharded_optimizer_bf16_mlp():
    cfg = dict(print_rank="none", widths=[64, 64, 64, 1], n_features=64, n_samples=256,
               dtype="bf16", nepochs=3, lr=1e-4)
    a = run_ranks(TrainConfig(device="cpu", shard_optimizer=True, **cfg), 2)
    b = run_ranks(TrainConfig(device="cpu", **cfg), 2)
    assert torch.equal(a[0]["final"], a[1]["final"])
    assert torch.equal(a[0]["final"], b[0]["final"])


def test_native_root_mode_is_accepted_by_config():
    from nnmpi_amd.utils.config import build_parser, config_from_args
    cfg = config_from_args(build_parser().parse_args(["--sync", "root", "--zero1"]))
    assert cfg.sync == "root" and cfg.shard_optimizer


def test_sharded_optimizer_checkpoint_resume_is_exact(tmp_path):
    """The checkpoint of a sharded run holds the re-assembled master AND momentum."""
    ck = str(tmp_path / "z.pt")
    cfg = dict(print_rank="none", shard_optimizer=True, n_samples=32)
    full = run_ranks(TrainConfig(device="cpu", nepochs=5, **cfg), 2)
    run_ranks(TrainConfig(device="cpu", nepochs=3, checkpoint=ck, **cfg), 2)
    res = run_ranks(TrainConfig(device="cpu", nepochs=5, resume=ck, **cfg), 2)
    assert torch.equal(res[0]["final"], full[0]["final"])


def test_zero1_checkpoint_resumes_at_another_world_size(tmp_path):
    """A ZeRO-1 checkpoint written at P=2 (arena padded to 2*64) resumes at P=3 -- with ZeRO-1
    (padded to 3*64) and without it: the momentum is stored per parameter name, unpadded, and
    re-laid into the new arena, so both resumed runs start from the saved state bit for bit and
    continue identically."""
    import torch as _t
    ck, ck2, ck3 = (str(tmp_path / n) for n in ("z.pt", "z3.pt", "a3.pt"))
    base = dict(print_rank="none", n_samples=48, scaling="global", averaging="weighted")
    run_ranks(TrainConfig(device="cpu", nepochs=3, checkpoint=ck, shard_optimizer=True, **base), 2)
    saved = _t.load(ck + ".train", weights_only=True)
    # resumed with nothing left to train: the re-saved state is the saved one
    run_ranks(TrainConfig(device="cpu", nepochs=3, resume=ck, checkpoint=ck2,
                          shard_optimizer=True, **base), 3)
    again = _t.load(ck2 + ".train", weights_only=True)
    for k, v in saved["momentum_by_name"].items():
        assert _t.equal(again["momentum_by_name"][k], v), k
        assert float(v.abs().sum()) > 0, k                  # a real (non-restarted) momentum
    a = run_ranks(TrainConfig(device="cpu", nepochs=5, resume=ck, shard_optimizer=True, **base), 3)
    b = run_ranks(TrainConfig(device="cpu", nepochs=5, resume=ck, checkpoint=ck3, **base), 3)
    assert _t.equal(a[0]["final"], b[0]["final"])


def test_resume_with_mismatched_optimizer_state_raises(tmp_path):
    ck = str(tmp_path / "m.pt")
    trainer.run_worker(TrainConfig(device="cpu", print_rank="none", nepochs=1, checkpoint=ck))
    import torch as _t
    st = _t.load(ck + ".train", weights_only=True)
    st["momentum_by_name"]["layers.0.weight"] = _t.zeros(4, 2)
    _t.save(st, ck + ".train")
    with pytest.raises(ValueError, match="layers.0.weight"):
        trainer.run_worker(TrainConfig(device="cpu", print_rank="none", nepochs=2, resume=ck))


def _reference_val_loss(res, n_val):
    """MSE of the final model on the held-out tail, recomputed independently with torch."""
    import numpy as np
    from sklearn.preprocessing import StandardScaler
    from nnmpi_amd.data import synth
    from nnmpi_amd.models.mlp import MLP
    X, y = synth.reference_regression()
    Xs = StandardScaler().fit_transform(X)
    Xv = torch.from_numpy(np.ascontiguousarray(Xs[-n_val:])).float()
    yv = torch.from_numpy(np.ascontiguousarray(y[-n_val:])).float().reshape(-1, 1)
    m = MLP()
    m.load_state_dict(res.state_dict)
    with torch.no_grad():
        return float(((m(Xv) - yv) ** 2).mean())


def test_validation_split_loss_matches_independent_eval():
    res = trainer.run_worker(TrainConfig(device="cpu", print_rank="none", val_fraction=0.25, nepochs=4))
    assert len(res.val_losses) == 4 and res.rows == 12
    assert res.val_losses[-1] == pytest.approx(_reference_val_loss(res, 4), rel=1e-5)


def test_validation_split_multirank_is_global():
    out = run_ranks(TrainConfig(device="cpu", print_rank="none", val_fraction=0.25, n_samples=32, nepochs=2), 2)
    assert [o["rows"] for o in out] == [12, 12]
    assert out[0]["losses"] != out[1]["losses"]        # local training losses differ
    assert out[0]["val"] == out[1]["val"] and len(out[0]["val"]) == 2   # one global value


def test_grad_accum_full_shard_equals_one_batch():
    """Cutting the whole-shard batch into 4 accumulated micro-batches gives the same steps
    (up to fp32 summation order) and the same per-epoch mean losses."""
    cfg = dict(print_rank="none", nepochs=5, n_samples=64, lr=0.01)
    a = trainer.run_worker(TrainConfig(device="cpu", **cfg))
    b = trainer.run_worker(TrainConfig(device="cpu", grad_accum=4, **cfg))
    assert a.steps == b.steps == 5
    torch.testing.assert_close(b.final_params, a.final_params, rtol=1e-5, atol=1e-6)
    assert b.losses == pytest.approx(a.losses, rel=1e-5)


def test_grad_accum_minibatches_multirank():
    """batch 4 x 2 accumulated micro-batches == batch 8 (same shuffled rows per step), on an
    uneven 3-rank split (9/8/8 rows) whose short shards run an empty last micro-batch."""
    cfg = dict(print_rank="none", nepochs=3, n_samples=25, lr=0.01)
    a = run_ranks(TrainConfig(device="cpu", batch_size=8, **cfg), 3)
    b = run_ranks(TrainConfig(device="cpu", batch_size=4, grad_accum=2, **cfg), 3)
    for x, y in zip(a, b):
        assert x["steps"] == y["steps"] == 3 * 2
        torch.testing.assert_close(y["final"], x["final"], rtol=1e-5, atol=1e-6)
    assert torch.equal(b[0]["final"], b[2]["final"])


def test_grad_accum_flag():
    from nnmpi_amd.utils.config import build_parser, config_from_args
    assert config_from_args(build_parser().parse_args(["--accum_steps", "3"])).grad_accum == 3
    with pytest.raises(ValueError):
        config_from_args(build_parser().parse_args(["--grad_accum", "0"]))


@pytest.mark.parametrize("fail_rank", [0, 1])
def test_one_rank_failure_ends_every_rank(fail_rank):
    """the reference hangs when one rank raises while the others block in
    gather/recv (ref.py:185,203).  Here 3 independently launched ranks (as mpiexec/torchrun
    would start them), one raising at epoch 1: every process must exit non-zero, well within
    timeout_s + 10 s (the collectives error out, or the watchdog aborts)."""
    import time
    timeout_s = 20
    port = _free_port()
    procs = []
    t0 = time.monotonic()
    for r in range(3):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="3", LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE="3", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   NNMPI_FAULT_INJECT=f"{fail_rank}:1", OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "dataParallelTraining_NN_MPI.py"),
             "--device", "cpu", "--nepochs", "50", "--timeout_s", str(timeout_s),
             "--print_rank", "none"],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    codes = []
    try:
        for p in procs:
            left = max(1.0, timeout_s + 10 - (time.monotonic() - t0) + 30)  # +30: python start
            p.wait(timeout=left)
            codes.append(p.returncode)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.monotonic() - t0
    assert all(c != 0 for c in codes), codes
    assert elapsed < timeout_s + 10 + 30, elapsed
    err = procs[fail_rank].stderr.read()
    assert "injected fault" in err


def test_profile_metrics_bus_bandwidth_from_comm_only(tmp_path):
    """--profile_steps: the per-phase times are labelled eager, and the bus bandwidth comes from
    the step's collectives timed alone (not from the join tail of the overlapped step)."""
    import json
    mj = str(tmp_path / "m.jsonl")
    run_ranks(TrainConfig(device="cpu", print_rank="none", metrics_json=mj, profile_steps=True,
                          widths=[64, 64, 1], n_features=64, n_samples=256), 2)
    lines = [json.loads(l) for l in open(mj)]
    prof = [l for l in lines if "profile_ms_per_step" in l]
    assert prof and prof[0]["phase_timing"] == "eager"
    assert prof[0]["comm_only_ms"] > 0 and prof[0]["comm_bus_GBps"] > 0


def test_row_chunk_buckets_cpu_bitwise(monkeypatch):
    """Layers cut into output-row chunk buckets (chunking forced on 512-wide layers) give the
    same parameters bit for bit as whole-layer buckets, at P=2 over gloo."""
    cfg = dict(print_rank="none", widths=[512, 512, 512, 1], n_features=512, n_samples=256,
               nepochs=2, lr=1e-4, data_gen="device", data_dist="local", scaling="none",
               bucket_mb=0.25)
    monkeypatch.setenv("NNMPI_CHUNK_MIN_TILES", "2")
    a = run_ranks(TrainConfig(device="cpu", **cfg), 2)
    monkeypatch.setenv("NNMPI_CHUNK_MIN_TILES", "100000")
    b = run_ranks(TrainConfig(device="cpu", **cfg), 2)
    assert torch.equal(a[0]["final"], a[1]["final"])
    assert torch.equal(a[0]["final"], b[0]["final"])
    from nnmpi_amd.engine.arena import Arena
    monkeypatch.setenv("NNMPI_CHUNK_MIN_TILES", "2")
    ar = Arena([(512, 512), (512, 512), (1, 512)], "meta", bucket_bytes=0.25 * 2 ** 20)
    assert ar.layer_chunks == {0: 2, 1: 2}
