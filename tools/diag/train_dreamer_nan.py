"""Pipelined vs sequential train_Agent epochs inside the fake-env train_dreamer
run (tests/test_gpu_api.py), from identical seeds: per-epoch losses."""
import os
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import test_gpu_api as T  # noqa: E402
from dreamer_amd import hip  # noqa: E402

dev = torch.device("cuda:0")
os.chdir(tempfile.mkdtemp())


def scenario(pipelined, recapture=False, no_wm=False, one_stream=False):
    print("=== pipelined" if pipelined else "=== sequential", "recapture" if recapture else "", "no_wm" if no_wm else "",
          flush=True)
    np.random.seed(0)
    d, _ = T._dreamer(dev, batch_size=4, sequence_length=16, horizon=5, buffer_size=256, random_iterations=2,
                      training_iterations=2, AC_epochs=2)
    hip.rng(dev).reseed(123)
    hip.adhoc(dev).reseed(456)
    eng = d.engine
    rm = eng.run_many

    def many(starts_list):
        if pipelined:
            if recapture and getattr(eng, "_pipe", None) is not None:
                eng._pipe["key"] = None
            if one_stream:
                orig = eng._pipe_capture

                def cap(key):
                    P = orig(key)
                    P["stream"] = torch.cuda.current_stream(dev)
                    return P
                eng._pipe_capture = cap
            r = rm(starts_list)
        else:
            out = []
            for s in starts_list:
                a, c = eng.run(s)
                out.append(torch.stack([a.reshape(()), c.reshape(())]).clone())
            r = torch.stack(out)
        print("  epochs:", r.tolist(), flush=True)
        return r
    eng.run_many = many
    if no_wm:
        d.train_world_model = lambda: [torch.zeros((), device=dev)]
    try:
        d.train_dreamer(T.FakeCarRacing(seed=1), T.FakeCarRacing(seed=2))
        print("  ok", flush=True)
    except AssertionError as e:
        print("  assert", e, flush=True)


import contextlib, io
res = {}
for mode in [True] * 12 + [False] * 6:
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(io.StringIO()):
        scenario(mode)
    lines = [l for l in buf.getvalue().splitlines() if "epochs" in l]
    key = lines[-1] if lines else "none"
    res.setdefault(("pipe" if mode else "seq", key), 0)
    res[("pipe" if mode else "seq", key)] += 1
for k, v in res.items():
    print(v, k, flush=True)
