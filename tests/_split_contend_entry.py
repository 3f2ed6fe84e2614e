"""One process of test_split_contention_gpu.py::test_split_step_two_processes_share_the_gpu:
a solo run of split steps, a file barrier with the other process, then the same steps again
while the other process runs its own.  Prints one JSON line {equal, errors, rows}."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    d, rank, rows = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    import torch
    import nnmpi_amd  # noqa: F401
    from test_split_contention_gpu import _run
    steps = 20

    def wait_for(name):
        t0 = time.monotonic()
        while not os.path.exists(os.path.join(d, name)):
            if time.monotonic() - t0 > 150:
                raise SystemExit(f"the other process never wrote {name}")
            time.sleep(0.005)
    # the solo runs one after the other (process 0 first), then both runs together
    if rank == 1:
        wait_for("solo0")
    solo = _run(rows, steps)
    open(os.path.join(d, f"solo{rank}"), "w").close()
    wait_for(f"solo{1 - rank}")
    errors = 0
    try:
        busy = _run(rows, steps)
    except RuntimeError as e:           # a timed-out hand-off wait (check_device_errors)
        print(e, file=sys.stderr)
        errors, busy = 1, None
    equal = busy is not None and all(torch.equal(a, b) for a, b in zip(solo[:4], busy[:4])) \
        and solo[4] == busy[4]
    diff = None
    if busy is not None and not equal:
        # where the runs part: the first step whose loss differs, and which state tensors differ
        k = next((i for i, (a, b) in enumerate(zip(solo[4], busy[4])) if a != b), None)
        diff = {"first_loss_step": k,
                "tensors": [n for n, a, b in zip(("master", "momentum", "shadow", "images"),
                                                  solo[:4], busy[:4]) if not torch.equal(a, b)]}
    print(json.dumps({"equal": bool(equal), "errors": errors, "rows": rows, "diff": diff}), flush=True)


if __name__ == "__main__":
    main()
