"""Experiment knobs: one switch decides whether they count.

Every ``NNMPI_*`` environment variable that changes WHAT runs -- a kernel variant, a schedule, a
transport, a split count -- is an experiment knob: honoured only when ``NNMPI_EXPERIMENTS=1``
(the native library checks the same switch, ``csrc/knobs.h``).  Without it a stray variable on
a benchmark box cannot silently change what is timed; ``bench.py`` reports every ``NNMPI_*``
variable it sees (and whether it was honoured) in its JSON line.

Operational variables (launcher plumbing, the supervisor's files, the native-library switch,
test fault injection) are not knobs: they do not select a code path of the training step.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

EXPERIMENTS = "NNMPI_EXPERIMENTS"

# variables that select code paths of the step (Python side and csrc/knobs.h)
KNOBS = {
    "NNMPI_ROWBAND": "row-band step schedule (0 off)",
    "NNMPI_ROWBAND_MIN_ROWS": "smallest batch that takes the row-band step",
    "NNMPI_RB_SPLITS": "row-band weight-gradient split-K slabs",
    "NNMPI_RB_PLAN": "row-band split-K plan (0 one launch, 1 phased; RowbandStep::plan)",
    "NNMPI_DEFER": "deferred bucket updates in weight-gradient epilogues (0 off)",
    "NNMPI_DEFER_WAIT": "deferred update waits per chunk / per layer",
    "NNMPI_CHUNK_MIN_TILES": "tiles per output-row chunk bucket",
    "NNMPI_BF16_REDUCE": "bf16 all-reduce algorithm (acc32 | rccl)",
    "NNMPI_F32_REDUCE": "fp32 all-reduce algorithm (ordered | rccl)",
    "NNMPI_SHM": "shared-memory all-reduce of CPU ranks (0: gloo)",
    "NNMPI_CPU_NATIVE": "native host step of tiny CPU models (0: PyTorch)",
    "NNMPI_STAGE_EPI": "LDS-staged 256x256 forward epilogue",
    "NNMPI_SGD_SERIAL": "SGD epilogue form",
    "NNMPI_PP_PREFETCH": "SGD-operand prefetch in the 256x256 weight gradient",
    "NNMPI_RB_BANDMAP": "XCD-contiguous band order of the row-band kernel",
    "NNMPI_RB_STORE": "row-band copy-out store policy (0 plain, 1 nt, 2 sc1)",
    "NNMPI_RB_SPLIT": "column-split row-band kernel for small batches: 0 off, 2 / 4 / 8 blocks per band, else auto",
    "NNMPI_RB_SPLIT_WAVES": "column-split row-band kernel: waves per block at 4 / 2 blocks per band (4 or 8)",
    "NNMPI_RB_WGSMALL": "small-batch row-band weight gradients: 1 un-split tiles with the update fused, 0 split-K slabs",
    "NNMPI_WGS_ASYNC": "small-batch weight-gradient LDS read mode (2 / 3 / 4, dma_gemm_tile ASYNC_TR)",
    "NNMPI_WGS_STAGES": "small-batch weight-gradient DMA ring stages (2 / 3 / 4 / 6 / 8)",
    "NNMPI_RB_FIXUP": "row-band split-K combine inside the weight-gradient launch (0: own launch)",
    "NNMPI_GEMM": "GEMM main loop (1 register-staged, 2 LDS-DMA)",
    "NNMPI_SLAB_STORE": "split-K slab store policy",
    "NNMPI_GROUP": "grouped backward launch (0 off)",
    "NNMPI_GRAPH_UPLOAD": "hipGraphUpload after instantiation (0 off)",
    "NNMPI_PAIR": "wide backward pair launches (experiments build)",
    "NNMPI_COMM_STANDIN": "k:gbps -- k CUs held after every bucket collective (standin.hip)",
    "NNMPI_WG_STAGES": "grouped weight-gradient launch DMA ring stages (default 2; 4)",
    "NNMPI_WG_REG": "register-staged operands in the grouped weight-gradient launch (A/B)",
    "NNMPI_WGM_ASYNC": "LDS read mode of the row-band weight-gradient launch (2; 3 pipelined)",
    "NNMPI_WGM_TILE": "row-band weight-gradient tile (0: 128x128, 8 waves; 1: 128x64, 4 waves)",
    "NNMPI_HEAD_BLOCKS": "block cap of the fused multi-output head (default 256)",
    "NNMPI_HEAD_FUSED": "multi-output head + weight gradient in one kernel (0: two launches)",
}

# plumbing, not knobs (never reported)
INTERNAL = {"NNMPI_SUPERVISED", "NNMPI_ATTEMPT", "NNMPI_PROGRESS_FILE", "NNMPI_RESULT_FILE",
            "NNMPI_LAUNCHER", "NNMPI_RDZV_KEY"}


def experiments() -> bool:
    return os.environ.get(EXPERIMENTS) == "1"


def knob(name: str, default: Optional[str] = None) -> Optional[str]:
    """The value of experiment knob ``name`` -- its default unless NNMPI_EXPERIMENTS=1."""
    assert name in KNOBS, name
    if not experiments():
        return default
    return os.environ.get(name, default)


def seen() -> Dict[str, dict]:
    """Every NNMPI_* variable in the environment (plumbing excluded): value and whether it took
    effect (knobs only with NNMPI_EXPERIMENTS=1; operational variables always)."""
    on = experiments()
    out = {}
    for k, v in sorted(os.environ.items()):
        if not k.startswith("NNMPI_") or k in INTERNAL:
            continue
        out[k] = {"value": v, "honoured": (on if k in KNOBS else True)}
    return out
