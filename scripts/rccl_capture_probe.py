"""Probe hipGraph capture of RCCL collectives at P=2 on ONE GPU (per-rank NCCL_HOSTID: the
ranks meet over RCCL's network transport on loopback).  Each variant runs in its own pair of
processes so a crash of one variant is contained.

    python scripts/rccl_capture_probe.py            # all variants, one JSON line each
"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, time
sys.path.insert(0, ROOT)
import torch
import torch.distributed as dist
import nnmpi_amd
from nnmpi_amd import native
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%s" % os.environ["PORT"],
                        rank=rank, world_size=world)
lib = native.lib()
obj = [lib.rccl_unique_id() if rank == 0 else None]
dist.broadcast_object_list(obj, src=0)
comm = native.make_comm(obj[0], world, rank, 0)
x = torch.full((1 << 16,), float(rank + 1), device="cuda")
s = torch.cuda.Stream()
variant = os.environ["VARIANT"]
capmode = int(os.environ.get("CAPMODE", "1"))
gs = lib.GradSync(comm, 1, int(os.environ.get("PRIO", "-1")))
tc = torch.cuda.Stream()
def body():
    h = int(s.cuda_stream)
    if variant == "inline":
        comm.allreduce(x.data_ptr(), x.numel(), 0, 0, h)
    elif variant == "torchside":
        x.mul_(1.0)
        tc.wait_stream(s)
        comm.allreduce(x.data_ptr(), x.numel(), 0, 0, int(tc.cuda_stream))
        s.wait_stream(tc)
    elif variant == "comm_origin":
        # capture ORIGIN = the comm stream; compute forks from it and joins back at the end
        s.wait_stream(tc)
        with torch.cuda.stream(s):
            x.mul_(1.0)
        tc.wait_stream(s)
        comm.allreduce(x.data_ptr(), x.numel(), 0, 0, int(tc.cuda_stream))
        s.wait_stream(tc)
        with torch.cuda.stream(s):
            x.mul_(1.0)
        comm.allreduce(x.data_ptr(), 64, 0, 0, int(tc.cuda_stream))   # a second one
        tc.wait_stream(s)
    elif variant == "side_then_inline":
        # a (dummy) collective issued on the ORIGIN stream first, then the side-stream one
        comm.allreduce(x.data_ptr(), 64, 0, 0, h)
        gs.bucket_ready(0, x.data_ptr(), x.numel(), 0, h)
        gs.join(h)
    else:
        x.mul_(1.0)                       # a kernel on the capture stream first
        gs.bucket_ready(0, x.data_ptr(), x.numel(), 0, h)
        gs.join(h)
with torch.cuda.stream(s):
    body(); s.synchronize()               # eager
    print("eager ok", float(x[0]), flush=True)
    g = lib.GraphRunner()
    origin = tc if variant == "comm_origin" else s
    g.begin(int(origin.cuda_stream), capmode)
    body()
    print("captured", flush=True)
    g.end()
    print("instantiated", flush=True)
    for _ in range(3):
        g.launch(int(s.cuda_stream))
    s.synchronize()
print("replayed ok", float(x[0]), flush=True)
dist.barrier()
del g, gs, comm
print("exit", flush=True)
os._exit(0)
'''


def run(variant, extra_env):
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", PORT=str(port), VARIANT=variant,
                   NCCL_HOSTID=f"probe-host-{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                   PYTHONFAULTHANDLER="1")
        env.update(extra_env)
        procs.append(subprocess.Popen([sys.executable, "-c", "ROOT=%r\n" % ROOT + CHILD], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    t0 = time.time()
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=max(1, 90 - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            p.kill()
            o, _ = p.communicate()
        outs.append((p.returncode, o))
    return {"variant": variant, "env": extra_env, "rc": [o[0] for o in outs],
            "stdout_r0": [l for l in outs[0][1].splitlines()
                          if not l.startswith("[") and "NCCL WARN" not in l][-12:]}


if __name__ == "__main__":
    cases = [("comm_origin", {}), ("inline", {}), ("side", {})]
    for v, e in cases:
        print(json.dumps(run(v, e)), flush=True)
