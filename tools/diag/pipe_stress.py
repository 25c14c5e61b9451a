"""Stress run_many (pipelined epochs) for run-to-run nondeterminism: from one
snapshot of the agent state, repeat the same 2-epoch call N times and compare
(and against the sequential epochs).  Config of tests/test_gpu_api.py's
train_dreamer drop-in test, with its world model trained a few steps."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import test_gpu_api as T  # noqa: E402
from formula import replay_data  # noqa: E402
from dreamer_amd import hip  # noqa: E402

dev = torch.device("cuda:0")
B = int(os.environ.get("PS_B", "4"))
d, _ = T._dreamer(dev, batch_size=B, sequence_length=16, horizon=5, buffer_size=256, AC_epochs=2)
fr, ac, rw, ct = replay_data(256, (64, 64), 3, seed=3)
d.buffer.load_arrays(fr, ac, rw, ct)
np.random.seed(0)
for _ in range(3):
    d.train_world_model()
eng = d.engine
ag = d.agent
ag.params_key()
state = lambda: [ag.fa.flat, ag.fc.flat, ag.ft.flat, ag.S_dev, eng.rng.state, ag.actor_optimiser.exp_avg,
                 ag.actor_optimiser.exp_avg_sq, ag.actor_optimiser.step_dev, ag.critic_optimiser.exp_avg,
                 ag.critic_optimiser.exp_avg_sq, ag.critic_optimiser.step_dev]
snap = [t.clone() for t in state()]
starts = [d.buffer.sample_start_indices(B) for _ in range(2)]


def restore():
    for t, s in zip(state(), snap):
        t.copy_(s)


scratch = torch.zeros(1 << 20, device=dev)


def run(pipe, poison=None, sync=False, value=float("nan")):
    restore()
    if poison is not None:
        poison.fill_(value)
    if sync:
        torch.cuda.synchronize()
    if pipe:
        r = eng.run_many(starts)
    else:
        r = torch.stack([torch.cat([x.reshape(1) for x in eng.run(s)]).clone() for s in starts])
    torch.cuda.synchronize()
    return r.cpu(), ag.fa.flat.cpu().clone()


ref, pa = run(False)
print("sequential", ref.tolist(), flush=True)
r, _ = run(True)
print("pipelined equal:", torch.equal(r, ref), flush=True)
P = eng._pipe
def persistent():
    out = {}
    for k, v in d.world_model.state_dict().items():
        out["wm." + k] = v
    for k, v in (d.buffer._dev or {}).items():
        out["ring." + k] = v
    for k, v in vars(eng).items():
        if isinstance(v, torch.Tensor):
            out["eng." + k] = v
    for k, v in hip.workspace(dev).bufs.items():
        out["ws." + k] = v
    return out


def poison(t):
    if t.is_floating_point():
        t.fill_(float("nan"))
    else:
        t.fill_(255 if t.dtype == torch.uint8 else -1)


def outcome(pipe, victim=None):
    restore()
    if victim is not None:
        poison(victim)
    r = eng.run_many(starts) if pipe else torch.stack(
        [torch.cat([x.reshape(1) for x in eng.run(s)]).clone() for s in starts])
    torch.cuda.synchronize()
    return r.cpu(), ag.fa.flat.cpu().clone(), ag.fc.flat.cpu().clone()


for pipe in (True, False):
    base = outcome(pipe)
    base2 = outcome(pipe)
    print("pipe" if pipe else "seq", "clean repeat equal:", all(torch.equal(x, y) for x, y in zip(base, base2)), flush=True)
    cands = dict(persistent())
    cands.update({"P.z0_1": P["z0"][1], "P.h0_1": P["h0"][1]})
    for k, t in cands.items():
        if k.startswith("wm.") or k.startswith("ring.") or k in ("eng.starts", "eng.rng"):
            continue
        o = outcome(pipe, t)
        ok = all(torch.equal(x, y) for x, y in zip(o, base))
        outcome(pipe)  # flush stale contents
        if not ok:
            print("  READ-BEFORE-WRITE?", "pipe" if pipe else "seq", k, o[0].tolist(), flush=True)
raise SystemExit
def slots():
    return [t.clone() for t in P["z0"] + P["h0"]]


run(True)
ref_slots = slots()
rngs = P["rng"].clone()
print("clean rerun slots equal:", [torch.equal(a, b) for a, b in zip((run(True), slots())[1], ref_slots)], flush=True)
for which in ("feat", "act_win", "z0_slot1", "none"):
    # replay the warm graph of slot 1 alone, on the main stream, from a fixed rng state
    t = dict(feat=eng.feat, act_win=eng.act_win, z0_slot1=P["z0"][1]).get(which)
    for sl in (0, 1):
        restore()
        eng.starts.copy_(torch.as_tensor(starts[sl], device=dev))
        P["rng"].copy_(rngs)
        if t is not None:
            t.fill_(float("nan"))
        P["graphs"][("warm", sl)].replay()
        torch.cuda.synchronize()
        z, h = P["z0"][sl], P["h0"][sl]
        print(f"warm slot {sl} alone, poison {which}: finite z {bool(torch.isfinite(z).all())} h {bool(torch.isfinite(h).all())}",
              f"feat finite {bool(torch.isfinite(eng.feat).all())} act_win finite {bool(torch.isfinite(eng.act_win).all())}",
              flush=True)
