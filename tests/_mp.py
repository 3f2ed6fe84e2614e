"""Multi-process helpers for CPU (gloo) tests: run ``run_worker(cfg)`` on N spawned ranks and
collect each rank's TrainResult through files (no shared state, separate RNGs)."""
import os
import socket
import tempfile

import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, cfg, outdir, fn_name):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    import nnmpi_amd  # noqa: F401
    from nnmpi_amd.engine import trainer
    res = getattr(trainer, fn_name)(cfg)
    torch.save({"losses": res.losses, "global_losses": res.global_losses, "val": res.val_losses,
                "final": res.final_params, "rows": res.rows, "steps": res.steps},
               os.path.join(outdir, f"r{rank}.pt"))


def run_ranks(cfg, world, fn_name="run_worker"):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_entry, args=(world, _free_port(), cfg, d, fn_name), nprocs=world,
                           join=True, start_method="spawn")
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
