"""Probe: AC_epochs = 2 with the pipelined epochs (engine.run_many) -- why the
side-stream warm start of epoch e+1 gains so little beside epoch e's chain.

Times K-epoch runs of run_many against K sequential engine.run epochs at
B = 256 under stream-priority settings of the warm stream and the main stream
(torch stream priorities; lower number = higher priority), and reports the
warm start's and the chain's own durations for reference.

  python tools/pipe_probe.py [K]
"""
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
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = 256
    _, d = bench.make_dreamer(bench.CAR_RACER, dev, B, 64, 15, 64, 1, 1, 0, None, "fp32")
    eng = d._engine
    rng = np.random.RandomState(3)
    starts = [rng.randint(0, 4096 - 64, size=B) for _ in range(K)]
    lo, hi = torch.cuda.Stream.priority_range()
    res = {"priority_range": [lo, hi]}

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best * 1e3 / K

    def seq():
        for s in starts:
            eng.run(s)

    res["sequential_ms_per_epoch"] = round(timed(seq), 4)
    # phases of one sequential epoch
    eng.run(starts[0], timing=True)
    torch.cuda.synchronize()
    res["phase_ms"] = {k: round(v, 4) for k, v in eng.phase_ms().items()}
    for name, wp, mp in (("default", None, None), ("warm_low", lo, None), ("warm_low_main_high", lo, hi),
                         ("main_high", None, hi)):
        eng._pipe = None  # recapture with fresh streams
        orig = torch.cuda.Stream

        def mk(device=None, priority=0, **kw):
            return orig(device=device, priority=priority, **kw)
        P = eng._pipe_capture((d.agent.params_key(), d.world_model.params_key(), d.buffer.device_key()))
        if wp is not None:
            P["stream"] = orig(device=dev, priority=wp)
        main = orig(device=dev, priority=mp) if mp is not None else torch.cuda.current_stream(dev)

        def pipe():
            with torch.cuda.stream(main):
                eng.run_many(starts)
        res[f"pipelined_{name}_ms_per_epoch"] = round(timed(pipe), 4)
        print(name, res[f"pipelined_{name}_ms_per_epoch"], flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
