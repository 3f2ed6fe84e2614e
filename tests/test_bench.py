"""bench.py contract: N ranks launched by the script itself, refusal to misreport, and the
BASELINE metric's derived fields (efficiency, exposed comm, overlap %, bus GB/s, strong scaling)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None, timeout=300):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
              "MASTER_PORT", "PMI_RANK", "PMI_SIZE", "OMPI_COMM_WORLD_RANK"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=timeout, env=e)


def _line(r):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout            # ONE JSON line on stdout, nothing else
    return json.loads(lines[0])


def test_bench_self_launches_two_ranks_cpu():
    d = _line(_run(["--gpus", "2", "--device", "cpu", "--config", "ref", "--steps", "10",
                    "--warmup", "2"]))
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["steps"] == 10 and d["warmup"] == 2
    assert d["config"]["comm"] == "gloo" and d["config"]["uneven_split"]
    assert d["config"]["global_batch"] == 31          # 16 * 2 - 1: the uneven split
    for k in ("parallel_efficiency", "exposed_comm_ms", "overlap_pct", "comm_bus_gbps",
              "comm_only_ms", "single_gpu_samples_per_s"):
        assert d[k] is not None, k
    assert 0.0 <= d["overlap_pct"] <= 100.0
    assert 0.0 < d["parallel_efficiency"]
    s = d["strong_scaling"]
    assert s["global_batch"] == 16 and s["samples_per_s"] > 0 and s["parallel_efficiency"] > 0


def test_bench_single_rank_cpu_unchanged_shape():
    d = _line(_run(["--device", "cpu", "--config", "ref", "--steps", "10", "--warmup", "2"]))
    assert d["n_gpus"] == 1 and d["config"]["parallelism"] == "dp1"
    assert d["config"]["comm"] == "none" and d["parallel_efficiency"] == 1.0
    assert d["strong_scaling"] is None


def test_bench_refuses_world_mismatch_under_launcher():
    r = _run(["--gpus", "3", "--device", "cpu", "--config", "ref", "--steps", "2"],
             env={"RANK": "0", "WORLD_SIZE": "2", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": "1"})
    assert r.returncode != 0 and "refusing" in r.stderr


def test_bench_rank_failure_fails_the_job():
    """A rank that dies makes the self-launched job exit non-zero (never a partial result)."""
    r = _run(["--gpus", "2", "--device", "cpu", "--config", "nonexistent"])
    assert r.returncode != 0


def test_bench_rank_sigsegv_relaunches_fresh_ranks():
    """A rank dying by a signal (what a crash inside a HIP/RCCL call looks like) does not cost the
    result: the supervisors kill the attempt's survivors and re-run the job in fresh processes
    with the inline schedule; the line says why (fallback) and which mode produced it."""
    d = _line(_run(["--gpus", "2", "--device", "cpu", "--config", "ref", "--steps", "6",
                    "--warmup", "2"], env={"NNMPI_BENCH_CRASH": "1:0"}))
    assert "SIGSEGV" in d["fallback"] and d["measured_mode"] == "--comm_mode inline"
    assert [e["result"] for e in d["attempts"]] == ["none", "full"]
    assert d["replicas_bitwise_equal"] is True and d["extras_error"] is None


def test_bench_rank_hang_is_detected_and_retried():
    """A rank that stops making progress (a peer blocked forever in a collective) is killed after
    the stall limit, and so is the rest of the attempt."""
    d = _line(_run(["--gpus", "3", "--device", "cpu", "--config", "ref", "--steps", "6",
                    "--warmup", "2"], env={"NNMPI_BENCH_HANG": "2:0", "NNMPI_BENCH_STALL_S": "8"}))
    assert "no progress" in d["fallback"] and d["attempts"][-1]["result"] == "full"
    assert d["n_gpus"] == 3 and d["replicas_bitwise_equal"] is True


def test_bench_crash_in_extras_keeps_the_measurement_under_torchrun():
    """Rank 0 dying after the timed region (inside the efficiency extras), under the driver's
    torchrun form: the timed measurement is still printed, with extras_error, and rc 0."""
    r = _torchrun(["--steps", "6", "--warmup", "2"],
                  env={"NNMPI_BENCH_CRASH": "0:0:extras single_gpu"})
    d = _line(r)
    assert d["extras_error"] and d["parallel_efficiency"] is None
    assert d["attempts"][0]["result"] == "core" and d["fallback"] is None
    assert d["value"] > 0 and d["replicas_bitwise_equal"] is True


def test_bench_every_attempt_failing_fails_the_job():
    r = _run(["--gpus", "2", "--device", "cpu", "--config", "ref", "--steps", "4", "--warmup",
              "1"], env={"NNMPI_BENCH_CRASH": "0:*"})
    assert r.returncode != 0 and r.stdout.strip() == ""
    assert r.stderr.count("injected SIGSEGV") == 2      # as launched, then inline


def test_scaling_report_arithmetic():
    from nnmpi_amd.utils.metrics import scaling_report
    # 4 ranks x 1000 rows; step 2.0 ms, compute-only 1.5 ms, collectives alone 1.0 ms
    r = scaling_report(4, 1000, 4000, 2.0, 1.5, 1.0, 3_000_000)
    assert r["samples_per_s"] == pytest.approx(4000 / 2e-3)
    assert r["single_gpu_samples_per_s"] == pytest.approx(1000 / 1.5e-3)
    assert r["parallel_efficiency"] == pytest.approx(0.75)        # = compute / step
    assert r["exposed_comm_ms"] == pytest.approx(0.5)
    assert r["overlap_pct"] == pytest.approx(50.0)                # 0.5 of 1.0 ms hidden
    assert r["comm_bus_gbps"] == pytest.approx(3.0)               # 3 MB / 1 ms
    # fully hidden / not hidden at all; clamped
    assert scaling_report(2, 10, 20, 1.0, 1.0, 0.4, 1)["overlap_pct"] == 100.0
    assert scaling_report(2, 10, 20, 3.0, 1.0, 0.4, 1)["overlap_pct"] == 0.0
    assert "overlap_pct" not in scaling_report(1, 10, 10, 1.0, 1.0, None, 0)


@pytest.mark.gpu
def test_bench_more_gpus_than_visible_fails():
    """On a box with fewer GPUs than --gpus the bench must exit non-zero, not run one rank."""
    import torch
    n = torch.cuda.device_count() + 1
    r = _run(["--gpus", str(n), "--steps", "2", "--warmup", "1"], timeout=120)
    assert r.returncode != 0
    assert "visible" in r.stderr
    assert r.stdout.strip() == ""


@pytest.mark.gpu
@pytest.mark.rowband
def test_bench_two_rank_rehearsal_on_one_gpu():
    """The whole multi-rank bench path -- tune of inline / ZeRO-1 / overlap schedules with the
    RCCL collectives captured in hipGraphs, timed region, efficiency / comm-only / strong-scaling
    extras -- with 2 RCCL ranks sharing the one GPU (NCCL_HOSTID rehearsal mode)."""
    r = _run(["--gpus", "2", "--shared_gpu_rehearsal", "--steps", "8", "--warmup", "2",
              "--tune_steps", "4"], timeout=300)
    d = _line(r)
    assert d["n_gpus"] == 2 and d["rccl_ranks"] == 2 and d["shared_gpu_rehearsal"]
    mode = d["config"]["comm_mode"]
    assert d["config"]["comm"] == "rccl" and mode.split("+")[0] in ("inline", "zero1", "overlap",
                                                                   "overlap_rowband", "inline_bf16")
    t = d["config"]["comm_tune_ms_per_step"]
    assert t is not None, (d.get("fallback"), d.get("attempts"))   # (measured by the tuner)
    assert {"inline", "zero1", "overlap", "overlap_rowband", "inline_bf16"} <= set(t)
    # the fp32-payload candidates and the bf16-payload inline one: under the two fastest
    # all-reduce schedules both algorithms (the default and the other one) are timed; the chosen
    # one is recorded (ZeRO-1 reduce-scatters: none)
    bf16 = mode.split("+")[0] == "inline_bf16"
    assert d["config"]["grad_dtype"] == ("bf16" if bf16 else "fp32")
    zero1 = mode == "zero1"
    alg = d["config"]["comm_tune_algorithm"]
    alts = [k for k in t if "+" in k]
    assert len(alts) == 2, t
    for k in alts:
        base, alt = k.split("+")
        assert base != "inline_bf16" and alt in ("rccl", "ordered") and alg[k] == alt != alg[base], (k, alg)
    if bf16:
        assert d["config"]["bf16_reduce"] == alg[mode] == "acc32", (mode, alg)
    else:
        assert d["config"]["f32_reduce"] == (None if zero1 else alg[mode]), (mode, alg)
    assert d["parallel_efficiency"] is not None and d["comm_bus_gbps"] is not None
    assert d["strong_scaling"]["global_batch"] == 8192
    assert d["final_loss"] == d["final_loss"]
    assert d["replicas_bitwise_equal"] is True and d["fallback"] is None


@pytest.mark.gpu
@pytest.mark.rowband
def test_bench_three_rank_rowband_uneven_rehearsal():
    """The bench's N > 1 shape at P = 3: 8192 * 3 - 1 rows split unevenly (8192, 8192, 8191), the
    row-band step (v2 images rebuilt after every multi-rank update) with the inline RCCL
    all-reduce, 3 RCCL ranks sharing the GPU: replicas bitwise equal."""
    r = _run(["--gpus", "3", "--shared_gpu_rehearsal", "--steps", "6", "--warmup", "2",
              "--comm_mode", "inline", "--no_extras"], timeout=300)
    d = _line(r)
    assert d["n_gpus"] == 3 and d["rccl_ranks"] == 3
    assert d["config"]["schedule"] == "rowband" and d["config"]["uneven_split"] is True
    assert d["config"]["global_batch"] == 8192 * 3 - 1
    assert d["replicas_bitwise_equal"] is True and d["final_loss"] == d["final_loss"]


@pytest.mark.gpu
def test_bench_tunes_the_bf16_reduction_algorithm():
    """A bf16 all-reduce payload (> 64 MB of fp32 gradient: the 2048-wide model) with chunk
    buckets forced, 3 RCCL ranks sharing the GPU: the tuner times every schedule with the
    one-rounding all-to-all (acc32) and the TWO fastest again with RCCL's own all-reduce (a slow
    default algorithm must not decide which schedule wins), reports all, keeps the fastest and
    records it; replicas bitwise equal."""
    r = _run(["--config", "wide2048", "--gpus", "3", "--shared_gpu_rehearsal", "--rows", "1024",
              "--chunk_tiles", "16", "--steps", "4", "--warmup", "2", "--tune_steps", "3",
              "--no_extras"], timeout=600)
    d = _line(r)
    t = d["config"]["comm_tune_ms_per_step"]
    assert d["config"]["grad_dtype"] == "bf16" and d["rccl_ranks"] == 3
    rccl = [k for k in t if k.endswith("+rccl")]
    assert len(rccl) == 2 and all(k[:-5] in t for k in rccl), t
    assert d["config"]["bf16_reduce"] == ("rccl" if d["config"]["comm_mode"].endswith("+rccl")
                                          else "acc32")
    if d["config"]["comm_mode"].startswith("overlap_c2"):
        # (the 2-chunks-per-layer candidate, --chunk_tiles 512: 2 chunk buckets per 2048-wide
        # layer's weight gradient)
        assert d["config"]["n_buckets"] > 1
    elif d["config"]["comm_mode"].startswith("overlap"):
        assert d["config"]["n_buckets"] > 5      # chunk buckets (inline replans to one bucket)
    assert d["replicas_bitwise_equal"] is True


@pytest.mark.gpu
@pytest.mark.rowband
def test_bench_driver_torchrun_form_on_one_gpu():
    """The driver's exact N-GPU launch (torch.distributed.run ... bench.py --gpus N) with the GPU
    ranks sharing the one device: per-rank supervisors under torchrun's agent store, RCCL ranks,
    one JSON line with replicas_bitwise_equal."""
    from nnmpi_amd.parallel.dist import free_port
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(free_port()), BENCH, "--gpus", "2", "--steps", "8", "--warmup", "2",
                        "--tune_steps", "4", "--shared_gpu_rehearsal"], capture_output=True,
                       text=True, timeout=300, env=e)
    d = _line(r)
    assert d["n_gpus"] == 2 and d["rccl_ranks"] == 2 and d["replicas_bitwise_equal"] is True
    assert d["fallback"] is None and d["attempts"][0]["result"] == "full"


@pytest.mark.gpu
def test_bench_gpu_rank_sigsegv_falls_back_to_inline():
    """The fallback with real GPU processes: RCCL rank 1 dies by SIGSEGV before the timed region
    (its peer holds an RCCL communicator and captured graphs); fresh ranks re-run the job with
    the inline schedule, and the replicas they leave are bitwise equal."""
    r = _run(["--gpus", "2", "--shared_gpu_rehearsal", "--steps", "8", "--warmup", "2",
              "--tune_steps", "4", "--no_extras"], env={"NNMPI_BENCH_CRASH": "1:0"}, timeout=300)
    d = _line(r)
    assert "SIGSEGV" in d["fallback"] and d["config"]["comm_mode"] == "inline"
    assert d["rccl_ranks"] == 2 and d["replicas_bitwise_equal"] is True


def _torchrun(args, n=2, env=None):
    from nnmpi_amd.parallel.dist import free_port
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
                           "--master-port", str(free_port()), BENCH, "--gpus", str(n), "--device",
                           "cpu", "--config", "ref"] + args, capture_output=True, text=True,
                          timeout=300, env=e)


def test_bench_under_torchrun_driver_command():
    """The driver's exact launch form: torch.distributed.run --nnodes=1 --nproc-per-node N
    --master-addr 127.0.0.1 --master-port P bench.py --gpus N (CPU plumbing here)."""
    d = _line(_torchrun(["--steps", "6", "--warmup", "2"]))
    assert d["n_gpus"] == 2 and d["steps"] == 6 and d["config"]["parallelism"] == "dp2"
    assert d["replicas_bitwise_equal"] is True and d["fallback"] is None


def test_bench_under_torchrun_sigsegv_falls_back():
    d = _line(_torchrun(["--steps", "6", "--warmup", "2"], n=3,
                        env={"NNMPI_BENCH_CRASH": "2:0:warm-up"}))
    assert "rank 2 killed by SIGSEGV" == d["fallback"] and d["n_gpus"] == 3


def test_bench_reports_and_ignores_a_stray_knob():
    """An experiment knob in the environment of a production run (no NNMPI_EXPERIMENTS=1) does
    not change what is timed -- the native library and the engine ignore it -- and the JSON line
    records it as not honoured; with NNMPI_EXPERIMENTS=1 it is recorded as honoured."""
    env = dict(os.environ, NNMPI_RB_SPLITS="7", NNMPI_ROWBAND="0")
    env.pop("NNMPI_EXPERIMENTS", None)
    r = subprocess.run([sys.executable, BENCH, "--device", "cpu", "--config", "ref", "--steps", "2",
                        "--warmup", "1", "--no_extras"], capture_output=True, text=True,
                       timeout=300, env=env)
    d = _line(r)
    k = d["knobs"]
    assert k["experiments"] is False
    assert k["env"]["NNMPI_RB_SPLITS"] == {"value": "7", "honoured": False}
    assert k["env"]["NNMPI_ROWBAND"]["honoured"] is False
    env["NNMPI_EXPERIMENTS"] = "1"
    r = subprocess.run([sys.executable, BENCH, "--device", "cpu", "--config", "ref", "--steps", "2",
                        "--warmup", "1", "--no_extras"], capture_output=True, text=True,
                       timeout=300, env=env)
    k = _line(r)["knobs"]
    assert k["experiments"] is True and k["env"]["NNMPI_RB_SPLITS"]["honoured"] is True


def test_native_set_knobs_need_the_experiments_switch():
    """The bindings' set_* kernel-selection knobs are ignored (return False) unless
    NNMPI_EXPERIMENTS=1 (csrc/knobs.h)."""
    code = ("from nnmpi_amd import native; l = native.lib(); "
            "print(l.experiments_on(), l.set_gemm_tile(64), l.set_pp256_order(0, 1))")
    env = dict(os.environ)
    env.pop("NNMPI_EXPERIMENTS", None)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                         env=env, cwd=os.path.dirname(BENCH)).stdout.split()
    assert out == ["False", "False", "False"]
    env["NNMPI_EXPERIMENTS"] = "1"
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                         env=env, cwd=os.path.dirname(BENCH)).stdout.split()
    assert out == ["True", "True", "True"]
