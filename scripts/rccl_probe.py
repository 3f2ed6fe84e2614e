"""Probe the RCCL paths on one GPU (each in its own subprocess so an abort is contained)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = {
    "native": r'''
import sys; sys.path.insert(0, ROOT)
import torch, nnmpi_amd
from nnmpi_amd import native
lib = native.lib()
print("rccl version", lib.rccl_version(), flush=True)
uid = lib.rccl_unique_id()
print("uid ok", len(uid), flush=True)
c = lib.RcclComm(uid, 1, 0, 0)
x = torch.ones(1024, device="cuda")
s = torch.cuda.current_stream()
c.allreduce(x.data_ptr(), x.numel(), 0, 0, s.cuda_stream)
torch.cuda.synchronize()
print("native allreduce ok", float(x.sum()), flush=True)
''',
    "torch": r'''
import torch, torch.distributed as dist
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29533", rank=0, world_size=1)
x = torch.ones(1024, device="cuda")
dist.all_reduce(x)
torch.cuda.synchronize()
print("torch nccl allreduce ok", float(x.sum()), flush=True)
dist.destroy_process_group()
''',
}

for name, code in CASES.items():
    env = dict(os.environ, NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,ENV")
    r = subprocess.run([sys.executable, "-c", "ROOT=%r\n" % ROOT + code], capture_output=True,
                       text=True, timeout=120, env=env)
    print(f"===== {name}: rc={r.returncode}")
    print(r.stdout[-3000:])
    print(r.stderr[-6000:])
