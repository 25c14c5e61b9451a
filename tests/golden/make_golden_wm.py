"""Golden fixtures for the world-model training step, made by running the
REFERENCE ``WorldModel.training_step`` (WorldModel.py:148-202).

Run in the build container only (``/root/reference`` does not exist on the GPU
box):  ``python tests/golden/make_golden_wm.py``.

For each configuration it builds the reference ``Dreamer``, fills its replay
``Buffer``, samples one batch with ``Buffer.sample_sequences`` under a fixed
``np.random`` seed and runs ``world_model.training_step`` twice from the same
weights:

* with ``torch.autocast`` disabled (fp32): the tight pin.  The gradients the
  optimiser sees (after clip_grad_norm_) and the post-AdamW parameters are
  recorded, and the Exp(1) draws behind each posterior sample are replayed from
  the same seed so the oracle (and the GPU path) can use them as explicit noise;
* as-is (fp16 autocast on the CPU): the loose check (total loss, post params).

On this CPU the reference's ``torch.amp.GradScaler()`` is disabled (no CUDA
device), so scale/unscale are the identity, exactly as they are in fp32.

Only data is written (inputs, noise, outputs, reduced-config weights).
"""
import contextlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
sys.path.insert(0, "/root/reference")

from formula import FULL, SMALL, replay_data  # noqa: E402
from make_golden import build_reference  # noqa: E402
from oracle import dreamer_oracle as O  # noqa: E402

# world-model fixtures at full width use a longer window than the AC ones
FULL_WM = dict(FULL)
FULL_WM.update(batch_size=3, horizon=6, sequence_length=8)
SMALL_WM = dict(SMALL)
SMALL_WM.update(batch_size=4, horizon=6, sequence_length=8)
SAMPLE = 997  # stride of the sampled entries kept for full-width tensors


@contextlib.contextmanager
def autocast_disabled():
    orig = torch.autocast

    def off(*a, **k):
        k["enabled"] = False
        return orig(*a, **k)

    torch.autocast = off
    try:
        yield
    finally:
        torch.autocast = orig


def _sampled(t):
    f = t.reshape(-1)
    return f[::SAMPLE].clone() if f.numel() > 4 * SAMPLE else f.clone()


def run_case(cfg, weights, n_fill, np_seed, torch_seed, full_grads):
    hw = tuple(cfg["observation_dims"])
    A = cfg["action_dims"]
    B, T = cfg["batch_size"], cfg["horizon"]
    R_, C_ = cfg["latent_state_dims"]
    frames, acts, rews, conts = replay_data(n_fill, hw, A, seed=0)

    def fresh():
        d = build_reference(cfg, weights)
        for i in range(n_fill):
            d.buffer.add_to_buffer(frames[i], acts[i], rews[i], conts[i])
        return d

    d = fresh()
    wm = d.world_model
    keys = ["world_model." + k for k, _ in wm.named_parameters()]
    sd0 = {k: v.detach().clone() for k, v in d.state_dict().items()}
    np.random.seed(np_seed)
    obs, act, rew, cont, _ = d.buffer.sample_sequences(batch_size=B)
    rec = {}
    ostep = wm.optimiser.step

    def step(*a, **k):
        rec["g"] = [p.grad.detach().clone() for p in wm.parameters()]
        return ostep(*a, **k)

    wm.optimiser.step = step
    torch.manual_seed(torch_seed)
    with autocast_disabled():
        total = wm.training_step(obs, act, rew, cont)
    sd1 = {k: v.detach().clone() for k, v in d.state_dict().items()}
    # the reference as shipped: fp16 autocast on the CPU
    d16 = fresh()
    torch.manual_seed(torch_seed)
    total16 = d16.world_model.training_step(obs, act, rew, cont)
    sd16 = {k: v.detach().clone() for k, v in d16.state_dict().items()}

    torch.manual_seed(torch_seed)
    q = torch.stack([torch.empty(B * R_, C_).exponential_() for _ in range(T)])
    np.random.seed(np_seed)
    starts = O.replay_starts(d.buffer.size, d.buffer.capacity, d.buffer.next_idx, cfg["sequence_length"], B)

    # ---- the oracle against the reference on the replayed noise ----
    P = {k: v.clone() for k, v in sd0.items()}
    for k in keys:
        P[k] = P[k].requires_grad_(True)
    o = O.wm_train_step(obs, act, rew, cont, P, q, R_, C_, T, keys,
                        (cfg["beta_prediction"], cfg["beta_dynamics"], cfg["beta_representation"]))
    assert torch.equal(o["total"].detach(), total.detach()), (float(o["total"]), float(total))
    maxg = max(float((a - b).abs().max()) for a, b in zip(o["grads_clipped"], rec["g"]))
    print(f"  total {float(total):.6f} (fp16 autocast {float(total16):.6f}); oracle grads max|d|={maxg:.3g}; "
          f"norm {float(o['norm']):.4f}")

    out = {
        "cfg_B": B, "cfg_S": cfg["sequence_length"], "cfg_H": T, "cfg_rows": R_, "cfg_cols": C_, "cfg_A": A,
        "buf_frames": d.buffer.observation_buffer, "buf_actions": d.buffer.action_buffer,
        "buf_rewards": d.buffer.reward_buffer, "buf_continues": d.buffer.continue_buffer,
        "buf_size": d.buffer.size, "buf_next_idx": d.buffer.next_idx, "buf_capacity": d.buffer.capacity,
        "np_seed": np_seed, "starts": starts.astype(np.int64), "q": q.numpy(),
        "total": total.detach().numpy(), "total_fp16": total16.detach().numpy(),
        "loss_pred": o["loss_pred"].detach().numpy(), "kl_dyn": o["kl_dyn"].detach().numpy(),
        "kl_rep": o["kl_rep"].detach().numpy(), "norm": o["norm"].numpy(),
        "hiddens": o["hiddens"].detach().numpy(), "latents": o["latents"].detach().numpy(),
        "post_logits": o["post_logits"].detach().numpy(),
        "wm_keys": np.array(keys),
    }
    for k, g in zip(keys, rec["g"]):
        out["grad_" + k] = g.numpy() if full_grads else _sampled(g).numpy()
        out["gnorm_" + k] = np.float32(float(g.norm()))
        out["post_" + k] = sd1[k].numpy() if full_grads else _sampled(sd1[k]).numpy()
        out["post16_" + k] = sd16[k].numpy() if full_grads else _sampled(sd16[k]).numpy()
    if weights != "formula":
        for k, v in sd0.items():
            out["param_" + k] = v.numpy()
    return out


def main():
    torch.set_num_threads(8)
    print("small config (reference default init)")
    np.savez_compressed(os.path.join(HERE, "small_wm.npz"), **run_case(SMALL_WM, "init", 74, 11, 12, True))
    print("full width (formula weights)")
    np.savez_compressed(os.path.join(HERE, "full_wm.npz"), **run_case(FULL_WM, "formula", 40, 13, 14, False))
    print("done")


if __name__ == "__main__":
    main()
