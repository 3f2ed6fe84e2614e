"""nnmpi_amd — MI355X-native data-parallel MLP training.

Capabilities mirror ``btourn/Neural-Networks-parallel-training-with-MPI``
(reference ``dataParallelTraining_NN_MPI.py``): a replicated MLP, a row-sharded synthetic
regression dataset, local forward/backward and per-step gradient averaging followed by
SGD-with-momentum.  The reference's gather-to-root / average / serial-send exchange
(ref.py:178-208) is replaced by a bucketed all-reduce (RCCL over xGMI on MI355X, gloo on CPU)
overlapped with backward; the hot path runs hand-written CDNA4 HIP kernels (``csrc/``).

Public surface (compatible with the reference):

* :func:`dist_train` — ``dist_train(args)`` with ``.lr .momentum .batch_size .nepochs``.
* :class:`MLP` — ``MLP()`` with attribute ``layers`` (``nn.Sequential``) and reference
  state_dict keys ``layers.{i}.weight/bias``.
* :class:`RegressionDataset` — ``RegressionDataset(X, y, scale_data=True)``.
"""
__version__ = "0.1.0"

from .models.mlp import MLP, MLPSpec  # noqa: E402,F401
from .data.dataset import RegressionDataset  # noqa: E402,F401
from .utils.config import TrainConfig, build_parser, config_from_args  # noqa: E402,F401


def dist_train(args):
    """Schedule a distributed training job (compat entry, reference ref.py:56).

    ``args`` may be an ``argparse.Namespace`` from :func:`build_parser` or any object with
    the reference attributes ``lr``, ``momentum``, ``batch_size``, ``nepochs``.
    Returns the :class:`~nnmpi_amd.engine.trainer.TrainResult` (the reference returns None).
    """
    from .engine.trainer import dist_train as _dt
    return _dt(args)
