"""Process runtime: rank discovery, rendezvous, self-spawn.

The reference relies on ``mpiexec`` + ``mpi4py`` (``README.md:12``, ``ref.py:8,61-63``).  mpi4py
is not available here, so the framework discovers its place in the job from the environment any
launcher leaves behind and rendezvouses through ``torch.distributed``'s C++ stores:

* MPICH/Hydra ``mpiexec``: ``PMI_RANK`` / ``PMI_SIZE`` / ``MPI_LOCALRANKID``;
* Open MPI ``mpirun``: ``OMPI_COMM_WORLD_RANK`` / ``_SIZE`` / ``_LOCAL_RANK``;
* ``torchrun`` / ``torch.distributed.run``: ``RANK`` / ``WORLD_SIZE`` / ``LOCAL_RANK`` +
  ``MASTER_ADDR``/``MASTER_PORT``;
* nothing: a single process, or ``--nprocs N`` self-spawns N local ranks.

Without ``MASTER_ADDR`` (plain ``mpiexec`` on one node) the rendezvous is a FileStore keyed by the
launcher's PID (all local ranks share their parent), so ``mpiexec -n N python
dataParallelTraining_NN_MPI.py`` works unchanged.  The control plane (metadata, barriers, the
RCCL unique-id exchange) always runs over gloo; the GPU data plane is RCCL.
"""
from __future__ import annotations

import datetime
import os
import socket
import sys
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class JobInfo:
    rank: int
    world: int
    local_rank: int
    local_world: int
    launcher: str           # "mpich" | "openmpi" | "torchrun" | "spawn" | "single"


def detect_job() -> JobInfo:
    env = os.environ
    if "PMI_RANK" in env and "PMI_SIZE" in env:
        return JobInfo(int(env["PMI_RANK"]), int(env["PMI_SIZE"]),
                       int(env.get("MPI_LOCALRANKID", env["PMI_RANK"])),
                       int(env.get("MPI_LOCALNRANKS", env["PMI_SIZE"])), "mpich")
    if "OMPI_COMM_WORLD_RANK" in env:
        return JobInfo(int(env["OMPI_COMM_WORLD_RANK"]), int(env["OMPI_COMM_WORLD_SIZE"]),
                       int(env.get("OMPI_COMM_WORLD_LOCAL_RANK", 0)),
                       int(env.get("OMPI_COMM_WORLD_LOCAL_SIZE", 1)), "openmpi")
    if "RANK" in env and "WORLD_SIZE" in env:
        return JobInfo(int(env["RANK"]), int(env["WORLD_SIZE"]), int(env.get("LOCAL_RANK", 0)),
                       int(env.get("LOCAL_WORLD_SIZE", env["WORLD_SIZE"])),
                       env.get("NNMPI_LAUNCHER", "torchrun"))
    return JobInfo(0, 1, 0, 1, "single")


def free_port() -> int:
    """A free TCP port for a rendezvous store, BELOW the kernel's ephemeral range (32768+ by
    default): an ephemeral port from bind(0) can be handed to another socket (an earlier job's
    RCCL / gloo bootstrap, a connection in TIME_WAIT) before rank 0's store binds it -- seen as
    EADDRINUSE in a multi-rank GPU test."""
    import random
    for _ in range(200):
        port = random.randint(20000, 32000)
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
            return port
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


_free_port = free_port


class _stdout_to_stderr:
    """fd-level redirect of stdout to stderr: gloo's C++ rendezvous prints "[Gloo] Rank r is
    connected to ..." on stdout, which would interleave with the reference's log lines and break
    one-JSON-line stdout contracts (bench.py)."""

    def __enter__(self):
        sys.stdout.flush()
        self._saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self._saved, 1)
        os.close(self._saved)
        return False


class ProcessGroupContext:
    """Owns the gloo control-plane group (and optionally a torch nccl group)."""

    def __init__(self, job: JobInfo, timeout_s: float = 300.0, want_nccl: bool = False,
                 device_id: Optional[int] = None):
        self.job = job
        self.rank, self.world = job.rank, job.world
        self.gloo = None
        self.nccl = None
        self.owned = False
        if job.world == 1 and not dist.is_initialized():
            return
        timeout = datetime.timedelta(seconds=timeout_s)
        if not dist.is_initialized():
            env = os.environ
            if "MASTER_ADDR" in env and "MASTER_PORT" in env:
                init = f"tcp://{env['MASTER_ADDR']}:{env['MASTER_PORT']}"
            else:
                key = env.get("NNMPI_RDZV_KEY", str(os.getppid()))
                init = f"file:///tmp/nnmpi_rdzv_{key}"
            with _stdout_to_stderr():
                dist.init_process_group("gloo", init_method=init, rank=job.rank,
                                        world_size=job.world, timeout=timeout)
            self.owned = True
        with _stdout_to_stderr():
            self.gloo = (dist.group.WORLD if dist.get_backend() == "gloo"
                         else dist.new_group(backend="gloo"))
            if want_nccl:
                self.nccl = dist.new_group(backend="nccl", timeout=timeout)

    def barrier(self):
        if self.gloo is not None:
            dist.barrier(group=self.gloo)

    def broadcast_object(self, obj, src: int = 0):
        if self.gloo is None:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.gloo)
        return lst[0]

    def allgather_object(self, obj):
        if self.gloo is None:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.gloo)
        return out

    def allreduce_cpu(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        if self.gloo is not None:
            dist.all_reduce(t, op=op, group=self.gloo)
        return t

    def destroy(self):
        if self.owned and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


def _spawn_entry(rank, world, fn, args, port, key):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port), "NNMPI_LAUNCHER": "spawn"})
    torch.set_num_threads(max(1, (os.cpu_count() or 1) // world))
    fn(*args)


def spawn(fn, nprocs: int, *args):
    """Run ``fn(*args)`` on ``nprocs`` local ranks (torch.multiprocessing, spawn start method)."""
    import torch.multiprocessing as mp
    port = _free_port()
    mp.start_processes(_spawn_entry, args=(nprocs, fn, args, port, str(os.getpid())),
                       nprocs=nprocs, join=True, start_method="spawn")


def under_launcher() -> bool:
    return detect_job().launcher != "single"


def log(msg: str):
    print(msg, file=sys.stderr, flush=True)
