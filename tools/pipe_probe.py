"""Probe: AC_epochs = 2 with the pipelined epochs (engine.run_many) -- how much
of the warm start of epoch e+1 hides beside epoch e's imagination / update.

One case per process (streams and HW queues of earlier cases would otherwise
share the device's few hardware queues and skew later ones):

  python tools/pipe_probe.py K CASE

CASE: "seq" (K sequential engine.run epochs), "pipe" (run_many as shipped),
"after:<fraction>" (sequential epochs timed before and after a pipelined run),
or "pipe:<warm CU fraction>:<chain priority>" -- the warm stream restricted
to that share of the CUs (engine.warm_stream; 1 = no mask) and the chain on a
stream of the given torch priority (0 = normal, -1 = high); an optional 4th
field sets DREAMER_WARM0_MAIN (1: the first warm start of a call on the chain's
stream over all CUs).  Prints one JSON
line: ms per epoch (best of 3 timed K-epoch runs at B = 256)."""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    case = sys.argv[2] if len(sys.argv) > 2 else "pipe"
    parts = case.split(":")
    if len(parts) > 1:
        os.environ["DREAMER_WARM_CUS"] = parts[1]
    if len(parts) > 2:
        os.environ["DREAMER_CHAIN_PRIORITY"] = parts[2]
    if len(parts) > 3:
        os.environ["DREAMER_WARM0_MAIN"] = parts[3]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = 256
    _, d = bench.make_dreamer(bench.CAR_RACER, dev, B, 64, 15, 64, 1, 1, 0, None, "fp32")
    eng = d._engine
    rng = np.random.RandomState(3)
    starts = [rng.randint(0, 4096 - 64, size=B) for _ in range(K)]

    def timed(fn, reps=max(3, 30 // K)):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best * 1e3 / K

    res = {"case": case, "K": K}
    if case.startswith("after"):
        # sequential epochs before and after a pipelined run in the same process:
        # does a CU-masked warm stream leave later work on the device slower?
        def seq():
            for s in starts:
                eng.run(s)
        res["seq_before_ms"] = round(timed(seq), 4)
        res["pipe_ms"] = round(timed(lambda: eng.run_many(starts)), 4)
        res["seq_after_ms"] = round(timed(seq), 4)
        res["warm_cus"] = os.environ.get("DREAMER_WARM_CUS")
        print(json.dumps(res), flush=True)
        return
    if case == "seq":
        def seq():
            for s in starts:
                eng.run(s)
        res["ms_per_epoch"] = round(timed(seq), 4)
        eng.run(starts[0], timing=True)
        torch.cuda.synchronize()
        res["phase_ms"] = {k: round(v, 4) for k, v in eng.phase_ms().items()}
    else:
        res["ms_per_epoch"] = round(timed(lambda: eng.run_many(starts)), 4)
        res["warm_cus"] = os.environ.get("DREAMER_WARM_CUS")
        res["chain_priority"] = os.environ.get("DREAMER_CHAIN_PRIORITY")
        res["warm0_main"] = os.environ.get("DREAMER_WARM0_MAIN")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
