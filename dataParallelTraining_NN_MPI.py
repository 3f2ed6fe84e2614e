"""Drop-in entry point with the reference's name and CLI.

    mpiexec -n N python dataParallelTraining_NN_MPI.py [--lr F] [--momentum F] [--batch_size N] [--nepochs N]

works as with the reference (README.md:12), and so do ``torchrun --nproc-per-node N ...`` and
``python dataParallelTraining_NN_MPI.py --nprocs N`` (self-spawn).  Extra flags select the GPU
path (``--device cuda``), presets, precision, scaling/averaging modes, checkpoints, etc.
(``--help``).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import nnmpi_amd  # noqa: E402
from nnmpi_amd.utils.config import build_parser  # noqa: E402

if __name__ == '__main__':
    parser = build_parser()
    args = parser.parse_args()
    nnmpi_amd.dist_train(args)
