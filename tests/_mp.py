"""Multi-process helpers for CPU (gloo) tests: run ``run_worker(cfg)`` on N spawned ranks and
collect each rank's TrainResult through files (no shared state, separate RNGs)."""
import os
import tempfile

import torch
import torch.multiprocessing as mp


def _free_port():
    from nnmpi_amd.parallel.dist import free_port
    return free_port()


def _entry(rank, world, port, cfg, outdir, fn_name):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    import nnmpi_amd  # noqa: F401
    from nnmpi_amd.engine import trainer
    res = getattr(trainer, fn_name)(cfg)
    torch.save({"losses": res.losses, "global_losses": res.global_losses, "val": res.val_losses,
                "final": res.final_params, "rows": res.rows, "steps": res.steps,
                "schedule": res.schedule},
               os.path.join(outdir, f"r{rank}.pt"))


def run_ranks(cfg, world, fn_name="run_worker"):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_entry, args=(world, _free_port(), cfg, d, fn_name), nprocs=world,
                           join=True, start_method="spawn")
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]


def run_ranks_proc(cfg: dict, world: int, env_per_rank=None, timeout: float = 150.0,
                   entry: str = "_rank_entry.py"):
    """Like :func:`run_ranks`, but every rank is an independent ``subprocess`` (as mpiexec /
    torchrun start them) with a hard time limit: on a hang or a failing rank every process is
    killed and the test fails with the ranks' stderr.  ``env_per_rank(rank) -> dict`` adds
    per-rank environment (e.g. RCCL settings for several ranks on one GPU)."""
    import json
    import subprocess
    import sys
    import time
    entry = os.path.join(os.path.dirname(os.path.abspath(__file__)), entry)
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        procs, logs = [], []
        for r in range(world):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                       LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=str(port), OMP_NUM_THREADS="1")
            if env_per_rank is not None:
                env.update(env_per_rank(r))
            log = open(os.path.join(d, f"r{r}.log"), "w+")
            logs.append(log)
            procs.append(subprocess.Popen([sys.executable, entry, json.dumps(cfg), d], env=env,
                                          stdout=log, stderr=subprocess.STDOUT))
        t0 = time.monotonic()
        failed = None
        try:
            while any(p.poll() is None for p in procs):
                if time.monotonic() - t0 > timeout:
                    failed = f"timeout after {timeout:.0f}s"
                    break
                bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
                if bad:
                    failed = f"rank exit codes {[p.returncode for p in procs]}"
                    break
                time.sleep(0.1)
            if failed is None and any(p.returncode != 0 for p in procs):
                failed = f"rank exit codes {[p.returncode for p in procs]}"
        finally:
            live = [p for p in procs if p.poll() is None]
            if live and failed:
                import signal
                for p in live:          # stack dump (faulthandler, _rank_entry.py), then kill
                    try:
                        p.send_signal(signal.SIGUSR1)
                    except OSError:
                        pass
                time.sleep(3)
            for p in procs:
                if p.poll() is None:
                    p.kill()
                    p.wait()
        if failed:
            out = []
            for r, log in enumerate(logs):
                log.seek(0)
                txt = log.read()
                # (RCCL's warning lines crowd out the stack dump: keep the Python frames)
                txt = "\n".join(l for l in txt.splitlines() if "NCCL WARN" not in l and l.strip())
                out.append(f"--- rank {r} ---\n" + txt[-6000:])
            raise AssertionError(failed + "\n" + "\n".join(out))
        for log in logs:
            log.close()
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
