"""One rank of a multi-process test job (started by ``_mp.run_ranks_proc``): reads the
TrainConfig fields as JSON, runs ``trainer.run_worker`` and saves the rank's results."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import faulthandler  # noqa: E402
import signal  # noqa: E402

# _mp.run_ranks_proc sends SIGUSR1 to a rank that hangs past its time limit before killing it:
# every thread's Python stack lands in the rank's log
faulthandler.register(signal.SIGUSR1, all_threads=True)

import torch  # noqa: E402

torch.set_num_threads(1)
import nnmpi_amd  # noqa: E402,F401
from nnmpi_amd.engine import trainer  # noqa: E402
from nnmpi_amd.utils.config import TrainConfig  # noqa: E402

cfg = TrainConfig(**json.loads(sys.argv[1]))
res = trainer.run_worker(cfg)
torch.save({"losses": res.losses, "global_losses": res.global_losses, "val": res.val_losses,
            "final": res.final_params, "rows": res.rows, "steps": res.steps,
            "schedule": res.schedule},
           os.path.join(sys.argv[2], f"r{res.rank}.pt"))
