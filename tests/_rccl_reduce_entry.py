"""One rank of the bf16-reduction numerics job (tests/test_multirank_gpu.py): every rank makes
a heavy-tailed fp32 "gradient" from its own seed, and the job reduces it three ways -- the
one-rounding bf16 all-reduce (RcclComm::allreduce_bf16_acc32), ncclAllReduce in bf16 and
ncclAllReduce in fp32 -- and saves the inputs and the three results."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import nnmpi_amd  # noqa: E402,F401
from nnmpi_amd import native  # noqa: E402
from nnmpi_amd.parallel import dist as pdist  # noqa: E402


def gradient(n: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    mag = torch.exp(2.0 * torch.randn(n, generator=g))        # magnitudes over many octaves
    return (torch.randn(n, generator=g) * mag).to(torch.float32)


def main():
    args = json.loads(sys.argv[1])
    outdir = sys.argv[2]
    job = pdist.detect_job()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    pg = pdist.ProcessGroupContext(job, 300.0)
    lib = native.lib()
    uid = pg.broadcast_object(lib.rccl_unique_id() if job.rank == 0 else None, 0)
    comm = native.make_comm(uid, job.world, job.rank, 0)
    n = int(args["n"])
    g = gradient(n, 1000 + job.rank)
    s = torch.cuda.current_stream()
    h = int(s.cuda_stream)
    acc = g.to(torch.bfloat16).to(dev)
    scratch = torch.empty(comm.acc32_scratch_elems(n), dtype=torch.bfloat16, device=dev)
    comm.allreduce_bf16_acc32(acc.data_ptr(), scratch.data_ptr(), n, h)
    ring = g.to(torch.bfloat16).to(dev)
    comm.allreduce(ring.data_ptr(), n, 1, 0, h)
    f32 = g.to(dev)
    comm.allreduce(f32.data_ptr(), n, 0, 0, h)
    s.synchronize()
    torch.save({"g": g, "acc32": acc.cpu(), "ring_bf16": ring.cpu(), "fp32": f32.cpu()},
               os.path.join(outdir, f"r{job.rank}.pt"))
    pg.barrier()
    del comm
    pg.destroy()


if __name__ == "__main__":
    main()
