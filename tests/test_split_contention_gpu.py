"""The column-split row-band kernel beside work that holds CUs (VERDICT r5 "Next" 3).

The blocks of one band wait for each other at every hand-off (csrc/kernels/rowband.hip
rowband_split_kernel), so the kernel is only correct if every band's blocks become resident
while it runs.  At P > 1 it shares the chip with communication kernels of the same process and,
in the shared-GPU rehearsal, with a second process's own split kernels.  These tests run the
split step (1,024 and 4,096-row shards of the 512-wide proxy: 8 and 2 blocks per band) while
other kernels hold CUs and check two things:

* no hand-off wait timed out (the sticky device error word, MLPEngine.check_device_errors), and
* the parameters, momentum, weight images and losses are bitwise equal to a solo run from the
  same initial state (the split step's summation orders do not depend on timing).

CU holders: (a) in-process, on a second stream -- a one-block spin kernel (torch's _sleep, one CU
held for ~100 us per step) plus a chain of bf16 GEMMs that keep every CU they get busy; (b) a
second PROCESS on the same GPU running the same split steps at the same time (each grid of 256
blocks competes with the other's).  The test has no stand-in of its own: the production library
alone runs it.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.rowband]

WIDTHS = [512, 512, 512, 512, 1]
HERE = os.path.dirname(os.path.abspath(__file__))


def _run(rows, steps, holder=None):
    """``steps`` fused-update split steps (eager) from a fixed init; ``holder(side_stream)`` is
    enqueued on a second stream before every step.  Returns the final state and the losses."""
    from nnmpi_amd.data import synth
    from nnmpi_amd.engine.arena import Arena
    from nnmpi_amd.engine.engine import MLPEngine
    from nnmpi_amd.models.mlp import MLPSpec, reference_init
    from nnmpi_amd.ops.hip_ops import HipOps
    from nnmpi_amd.parallel.sync import NoSync
    spec = MLPSpec(tuple(WIDTHS), "relu", "mse")
    ar = Arena([spec.layer_shape(i) for i in range(spec.n_layers)], "cuda",
               shadow_dtype=torch.bfloat16)
    ar.bind_model(reference_init(WIDTHS, "relu", seed=5))
    eng = MLPEngine(spec, ar, HipOps("cuda"), NoSync(ar), device="cuda", dtype=torch.bfloat16,
                    rows_capacity=rows, lr=1e-5, momentum=0.9, use_graph=False)
    X, Y = synth.chunked_regression(0, rows, WIDTHS[0], out=1, device="cuda")
    eng.load_batch(X.to(torch.bfloat16), Y)
    eng.set_scales(1.0 / rows, 1.0 / rows, 1.0)
    assert eng.uses_rowband_split(rows)
    side = torch.cuda.Stream()
    losses = []
    for _ in range(steps):
        if holder is not None:
            holder(side)
        eng.step()
        losses.append(eng.loss())        # (host sync + the error word: raises on a timeout)
    eng.synchronize()
    torch.cuda.synchronize()
    # (a diverging run would compare NaN with NaN -- never equal: the rate keeps it finite)
    assert all(l == l and abs(l) < 1e30 for l in losses), losses
    return (ar.master.clone(), ar.momentum.clone(), ar.shadow.clone(), eng._rb_buf.clone(), losses)


def _holder(gemms: int, spin_cycles: int):
    """Work on the side stream that holds CUs while the next step runs: one spinning block and a
    chain of bf16 GEMMs (each reads the previous one's output, so they run back to back)."""
    a = torch.randn(2048, 2048, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(2048, 2048, device="cuda", dtype=torch.bfloat16) * 0.02

    def hold(side):
        with torch.cuda.stream(side):
            torch.cuda._sleep(spin_cycles)
            x = a
            for _ in range(gemms):
                x = x @ b
    return hold


@pytest.mark.parametrize("rows", [1024, 4096])
def test_split_step_beside_cu_holding_stream(rows, monkeypatch):
    monkeypatch.setenv("NNMPI_ROWBAND_MIN_ROWS", "6144")   # (the production threshold)
    solo = _run(rows, 6)
    for gemms, spin in ((0, 200_000), (8, 200_000), (32, 50_000)):
        busy = _run(rows, 6, _holder(gemms, spin))
        for x, y in zip(solo[:4], busy[:4]):
            assert torch.equal(x, y), (gemms, spin)
        assert solo[4] == busy[4]


def test_split_step_two_processes_share_the_gpu(tmp_path):
    """Two processes run split steps on one GPU at the same time (each after a solo run of its
    own): no timed-out wait, and each concurrent run bitwise equals its solo run."""
    entry = os.path.join(HERE, "_split_contend_entry.py")
    env = dict(os.environ, NNMPI_ROWBAND_MIN_ROWS="6144", NNMPI_EXPERIMENTS="1",
               PYTHONPATH=os.path.dirname(HERE) + os.pathsep + os.environ.get("PYTHONPATH", ""))
    procs = [subprocess.Popen([sys.executable, entry, str(tmp_path), str(r), rows], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r, rows in enumerate(("1024", "4096"))]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=240)
            outs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]
        res = json.loads(out.strip().splitlines()[-1])
        assert res["equal"] and res["errors"] == 0, res
