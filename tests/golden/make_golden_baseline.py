"""Reference-run fixture at BASELINE.json configs[0]'s shape (CarRacing widths,
B=16, S=50, H=15) with the return normaliser above 1 (S0 = 5).

Run in the build container only (``/root/reference`` does not exist on the GPU
box):  ``python tests/golden/make_golden_baseline.py``.

It runs the reference's train_Agent unit of work exactly as make_golden.py's
``run_case`` does (sample_sequences -> warm_start_generator -> dream_episodes
-> train_step, Dreamer.py:264-287; weights from formula.py) and checks the
oracle reproduces it bit-for-bit from the replayed noise.  The fixture is kept
compact: the replay frames and the noise are NOT stored, because both are
regenerated deterministically by the tests (``formula.replay_data`` with
numpy's PCG64, and ``torch.manual_seed(torch_seed)`` followed by the
reference's draw order: S/2 x exponential_, then H x (normal_, exponential_));
a checksum of the frames and of every noise tensor pins that regeneration.
Latents are stored as class indices; gradients and post-step parameters as
every 61st element plus the per-tensor L2 norms (full tensors below 4096
elements).  Only data is written; no reference source is copied.
"""
import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import run_case  # noqa: E402  (imports the reference from /root/reference)
from formula import FULL  # noqa: E402

BASE = dict(FULL)
BASE.update(batch_size=16, sequence_length=50, horizon=15, buffer_size=96)
N_FILL, NP_SEED, TORCH_SEED, S0 = 80, 11, 12, 5.0
STRIDE, SMALL_T = 61, 4096


def digest(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()[:8], dtype=np.int64)[0]


def sampled(a):
    a = np.asarray(a, dtype=np.float32).reshape(-1)
    return a if a.size < SMALL_T else a[::STRIDE].copy()


def main():
    torch.set_num_threads(8)
    full = run_case(BASE, "formula", N_FILL, NP_SEED, TORCH_SEED, S0=S0)
    C = int(full["cfg_cols"])
    out = {k: full[k] for k in ("cfg_B", "cfg_S", "cfg_H", "cfg_rows", "cfg_cols", "cfg_A", "buf_size",
                                "buf_next_idx", "buf_capacity", "np_seed", "starts", "buf_actions", "buf_rewards",
                                "buf_continues", "h0", "hiddens", "actions", "rewards", "continues", "mus",
                                "sigmas", "R", "loss_actor", "loss_critic", "S_after")}
    out.update(torch_seed=np.int64(TORCH_SEED), S0=np.float32(S0), n_fill=np.int64(N_FILL),
               sample_stride=np.int64(STRIDE), small_tensor=np.int64(SMALL_T))
    out["frames_digest"] = digest(full["buf_frames"])
    for k in ("q_warm", "eps", "q"):
        out[k + "_digest"] = digest(full[k])
    out["z0_idx"] = full["z0"].reshape(-1, C).argmax(-1).astype(np.int8)
    out["latents_idx"] = full["latents"].reshape(-1, C).argmax(-1).astype(np.int8)
    for k in list(full):
        if k.startswith("gradc_agent.") or k.startswith("post_agent."):
            out[k] = sampled(full[k])
            out["norm_" + k] = np.float32(np.linalg.norm(full[k].astype(np.float64)))
    np.savez_compressed(os.path.join(HERE, "baseline_b16.npz"), **out)
    print("wrote baseline_b16.npz")


if __name__ == "__main__":
    main()
