"""Per-rank job supervisor with coordinated, fresh-process retries.

The reference has no answer to a rank dying: ``mpiexec`` either tears the whole job down or,
when one rank raises while the others block in ``comm.gather`` / ``comm.recv``, the job hangs
(``ref.py:185,203``).  A GPU job can also die in ways no Python ``except``
sees -- a SIGSEGV inside a driver call such as ``hipStreamEndCapture`` of an RCCL collective
(profiles/r2_experiments.md §6) -- and one dead rank leaves its peers spinning inside a captured
collective.

Each launched rank (torchrun worker, self-spawned rank, ``mpiexec`` process) therefore runs as a
*supervisor* that never touches the GPU.  It starts the real rank as a child process (a new
process, never an ``exec``), and the supervisors agree on every attempt's outcome through a TCP
store:

* a child that exits non-zero, dies by a signal, or makes no progress for ``stall_s`` seconds
  (the child touches its progress file at every milestone) marks the attempt failed;
* every supervisor that sees the failure kills its own child, so no peer stays blocked;
* the attempt's result is whatever rank 0's child left in its result file (``full``: the whole
  JSON line; ``core``: the timed measurement before the post-run extras; ``none``);
* with no result, every supervisor starts attempt k+1 together, with the next, more
  conservative arguments (fresh processes, fresh rendezvous port, fresh communicator).

Rank 0's supervisor prints the one result line (annotated with the attempts and the reason of
any fallback), then all supervisors exit with one agreed code, so a launcher that kills the
job on the first non-zero exit (torchrun) never cuts the line off.
"""
from __future__ import annotations

import datetime
import json
import os
import signal
import subprocess
import sys
import tempfile
import time
from typing import Callable, List, Optional

ENV_SUPERVISED = "NNMPI_SUPERVISED"
ENV_PROGRESS = "NNMPI_PROGRESS_FILE"
ENV_RESULT = "NNMPI_RESULT_FILE"
ENV_ATTEMPT = "NNMPI_ATTEMPT"
# exit code of a child whose work finished but whose teardown stalled (bench._exit_watchdog)
RC_TEARDOWN_STALL = 4


def progress(phase: str):
    """Called by a supervised child at every milestone: the supervisor's stall detector sees the
    file's mtime move.  A no-op without a supervisor."""
    path = os.environ.get(ENV_PROGRESS)
    if path:
        try:
            with open(path, "w") as f:
                f.write(f"{time.time():.3f} {phase}\n")
        except OSError:
            pass


def write_result(obj: dict):
    """Atomically (re)write the child's result (rank 0's is the job's line)."""
    path = os.environ.get(ENV_RESULT)
    if not path:
        return
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
    os.replace(tmp, path)


def supervised() -> bool:
    return os.environ.get(ENV_SUPERVISED) == "1"


def _describe(rc: int) -> str:
    if rc < 0:
        try:
            return f"killed by {signal.Signals(-rc).name}"
        except ValueError:
            return f"killed by signal {-rc}"
    return f"exit code {rc}"


def rendezvous_shared(world: int, local_world: int) -> bool:
    """The supervisors of every rank can meet: a TCP store (MASTER_ADDR / MASTER_PORT), or all
    ranks on this node (the FileStore of their common launcher)."""
    env = os.environ
    return ("MASTER_ADDR" in env and "MASTER_PORT" in env) or local_world == world


def _launcher_key() -> str:
    """A per-job key for the FileStore path when there is no MASTER_*: the launcher's pid plus its
    start time (a pid reused by a later launcher gets a different key, so a file left behind by
    a crashed job is never picked up), or the launcher's job id when it exports one."""
    env = os.environ
    for k in ("NNMPI_RDZV_KEY", "PMIX_NAMESPACE", "OMPI_MCA_ess_base_jobid", "PMI_KVSNAME",
              "SLURM_JOB_ID"):
        if env.get(k):
            return "".join(c if c.isalnum() else "_" for c in f"{k}_{env[k]}")[:96]
    ppid = os.getppid()
    start = "0"
    try:
        with open(f"/proc/{ppid}/stat") as f:
            start = f.read().rsplit(")", 1)[1].split()[19]   # field 22: starttime
    except (OSError, IndexError):
        pass
    return f"{ppid}_{start}"


def _make_store(rank: int, world: int, timeout_s: float):
    import torch.distributed as dist
    env = os.environ
    timeout = datetime.timedelta(seconds=timeout_s)
    agent = env.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true"
    if "MASTER_ADDR" in env and "MASTER_PORT" in env:
        # torchrun's agent already serves a store on MASTER_PORT: join it as a client;
        # otherwise (bench.py's own spawn) rank 0 serves it there
        st = dist.TCPStore(env["MASTER_ADDR"], int(env["MASTER_PORT"]), world,
                           is_master=(rank == 0 and not agent), timeout=timeout,
                           wait_for_workers=False)
    else:   # plain mpiexec on one node: the ranks share their launcher (rendezvous_shared)
        st = dist.FileStore(os.path.join(tempfile.gettempdir(), f"nnmpi_sup_{_launcher_key()}"),
                            world)
        st.set_timeout(timeout)
    restart = env.get("TORCHELASTIC_RESTART_COUNT", "0")
    return dist.PrefixStore(f"nnmpi_supervisor/{restart}", st)


class Supervisor:
    """Run ``attempts[k]`` (an argv list per attempt) as this rank's child, k = 0, 1, ...
    until one leaves a result; see the module docstring."""

    def __init__(self, rank: int, world: int, stall_s: float = 300.0, store_timeout_s: float = 900.0,
                 poll_s: float = 0.2, kill_grace_s: float = 10.0):
        self.rank, self.world = rank, world
        self.stall_s = float(stall_s)
        self.poll_s = poll_s
        self.kill_grace_s = kill_grace_s
        self.store = _make_store(rank, world, store_timeout_s)
        self.child: Optional[subprocess.Popen] = None
        self._tmp = tempfile.mkdtemp(prefix=f"nnmpi_sup_r{rank}_")
        signal.signal(signal.SIGTERM, self._on_term)

    # -- child control ----------------------------------------------------------------------
    def _on_term(self, signum, frame):
        self._kill_child()
        os._exit(128 + signum)

    def _kill_child(self):
        p = self.child
        if p is None or p.poll() is not None:
            return
        try:
            p.terminate()
            p.wait(timeout=self.kill_grace_s)
        except subprocess.TimeoutExpired:
            p.kill()
            try:
                p.wait(timeout=self.kill_grace_s)
            except subprocess.TimeoutExpired:
                pass
        except OSError:
            pass

    def _count(self, key: str, inc: int = 0) -> int:
        return int(self.store.add(key, inc))

    def _wait_count(self, key: str, n: int, timeout_s: float) -> bool:
        t0 = time.monotonic()
        while self._count(key) < n:
            if time.monotonic() - t0 > timeout_s:
                return False
            time.sleep(self.poll_s)
        return True

    # -- one attempt ------------------------------------------------------------------------
    def _attempt(self, k: int, argv: List[str], env_extra: dict):
        """Run attempt k; returns (result_state, own_failure, all_failures)."""
        r, st = self.rank, self.store
        from .dist import free_port
        if r == 0:
            st.set(f"a{k}/port", str(free_port()))
        port = st.get(f"a{k}/port").decode()
        prog = os.path.join(self._tmp, f"progress_{k}")
        res = os.path.join(self._tmp, f"result_{k}.json")
        env = dict(os.environ)
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)   # the child's rank 0 serves its own store
        env.update(env_extra)
        env.update({ENV_SUPERVISED: "1", ENV_PROGRESS: prog, ENV_RESULT: res, ENV_ATTEMPT: str(k),
                    "MASTER_ADDR": os.environ.get("MASTER_ADDR", "127.0.0.1"),
                    "MASTER_PORT": port})
        progress_mark = None
        last_move = time.monotonic()
        self.child = subprocess.Popen(argv, env=env)
        own = None
        while True:
            rc = self.child.poll()
            if rc is not None:
                if rc != 0:
                    own = f"rank {r} {_describe(rc)}"
                    if rc == RC_TEARDOWN_STALL:
                        own += " (teardown stalled)"
                break
            if self._count(f"a{k}/nfail") > 0:
                self._kill_child()          # a peer failed: ours cannot finish either
                break
            try:
                m = os.stat(prog).st_mtime_ns
            except OSError:
                m = None
            now = time.monotonic()
            if m != progress_mark:
                progress_mark, last_move = m, now
            elif now - last_move > self.stall_s:
                own = f"rank {r} made no progress for {self.stall_s:.0f} s"
                self._kill_child()
                break
            time.sleep(self.poll_s)
        if own is not None:
            st.set(f"a{k}/fail/{r}", own)
            self._count(f"a{k}/nfail", 1)
        if r == 0:
            state = "none"
            try:
                with open(res) as f:
                    state = "full" if json.load(f).get("complete") else "core"
            except (OSError, ValueError):
                pass
            st.set(f"a{k}/result", state)
        self._count(f"a{k}/ended", 1)
        # every peer either finishes or is killed within stall_s + the kill grace; a peer that
        # never reports fails the attempt (its result key may never be written)
        if not self._wait_count(f"a{k}/ended", self.world, self.stall_s + 4 * self.kill_grace_s + 60):
            return "none", own, [f"rank {r}: peers did not end attempt {k} in time"], res
        state = st.get(f"a{k}/result").decode()
        fails = []
        if self._count(f"a{k}/nfail") > 0:
            for q in range(self.world):
                if st.check([f"a{k}/fail/{q}"]):
                    fails.append(st.get(f"a{k}/fail/{q}").decode())
        return state, own, fails, res

    def run(self, attempts: List[List[str]], describe: Callable[[int], str],
            annotate: Optional[Callable[[dict, list], dict]] = None, env_extra=None) -> int:
        """Run the attempts; rank 0 prints the result line.  Returns the agreed exit code."""
        log = []
        line, code = None, 1
        for k, argv in enumerate(attempts):
            state, own, fails, res = self._attempt(k, argv, env_extra or {})
            log.append({"attempt": k, "mode": describe(k), "result": state,
                        "failures": fails or None})
            for f in (fails if self.rank == 0 else []):
                print(f"[supervisor] attempt {k} ({describe(k)}): {f}", file=sys.stderr,
                      flush=True)
            if state != "none":
                if self.rank == 0:
                    with open(res) as f:
                        line = json.load(f)
                    line.pop("complete", None)
                # finished measurement whose teardown stalled: still a defect -> non-zero
                code = RC_TEARDOWN_STALL if (fails and state == "full" and any(
                    "teardown stalled" in x for x in fails)) else 0
                break
        if self.rank == 0:
            if line is not None:
                if annotate is not None:
                    line = annotate(line, log)
                print(json.dumps(line), flush=True)
            self.store.set("final_rc", str(code))
        code = int(self.store.get("final_rc").decode())
        self._count("printed", 1)
        self._wait_count("printed", self.world, 60)
        # rank 0 may serve the store: it leaves last, after every peer's final store call
        if self.rank == 0:
            self._wait_count("bye", self.world - 1, 60)
        else:
            self._count("bye", 1)
        return code
