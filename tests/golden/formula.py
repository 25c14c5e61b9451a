"""Deterministic closed-form weights and configs shared by the fixture
generator (``make_golden.py``) and the tests, so full-width fixtures need no
committed weight file.  Test infrastructure only."""
import math

import numpy as np
import torch

# reduced-width configuration (SURVEY.md §8c golden-vector recipe)
SMALL = dict(
    hidden_state_dims=64, latent_state_dims=[8, 8], action_dims=3, observation_dims=[32, 32],
    encoder_filter_num_1=8, encoder_filter_num_2=16, encoder_hidden_layer_nodes=32,
    decoder_filter_num_1=8, decoder_filter_num_2=16, decoder_hidden_layer_nodes=32,
    dyn_pred_hidden_num_nodes_1=32, dyn_pred_hidden_num_nodes_2=32,
    rew_pred_hidden_num_nodes_1=32, rew_pred_hidden_num_nodes_2=32,
    cont_pred_hidden_num_nodes_1=32, cont_pred_hidden_num_nodes_2=32,
    hidden_layer_actor_1_size=32, hidden_layer_actor_2_size=32,
    hidden_layer_critic_1_size=32, hidden_layer_critic_2_size=32,
    critic_reward_buckets=255, device="cpu",
    horizon=5, batch_size=4, nu=0.0003, lambda_=0.95, gamma=0.99, buffer_size=64,
    sequence_length=8, seed=42, training_iterations=1, random_iterations=1,
    actor_lr=0.00008, actor_betas=[0.9, 0.999], actor_eps=0.00001,
    critic_lr=0.0001, critic_betas=[0.9, 0.999], critic_eps=0.00001, AC_epochs=1,
    world_model_lr=0.0001, world_model_betas=[0.9, 0.999], world_model_eps=0.00001, WM_epochs=1,
    beta_prediction=1.0, beta_dynamics=0.5, beta_representation=0.1,
)

# full width (car_racer_config.yaml) with small batch/horizon for fixtures
FULL = dict(SMALL)
FULL.update(
    hidden_state_dims=600, latent_state_dims=[32, 32], observation_dims=[64, 64],
    encoder_filter_num_1=32, encoder_filter_num_2=64, encoder_hidden_layer_nodes=200,
    decoder_filter_num_1=32, decoder_filter_num_2=64, decoder_hidden_layer_nodes=200,
    dyn_pred_hidden_num_nodes_1=200, dyn_pred_hidden_num_nodes_2=200,
    rew_pred_hidden_num_nodes_1=200, rew_pred_hidden_num_nodes_2=200,
    cont_pred_hidden_num_nodes_1=200, cont_pred_hidden_num_nodes_2=200,
    hidden_layer_actor_1_size=200, hidden_layer_actor_2_size=200,
    hidden_layer_critic_1_size=200, hidden_layer_critic_2_size=200,
    horizon=3, batch_size=2, sequence_length=4, buffer_size=64,
)


def formula_tensor(shape, key_index, kind):
    n = int(np.prod(shape)) if len(shape) else 1
    i = torch.arange(n, dtype=torch.float64)
    s = torch.sin(1.7 * i + 0.37 * key_index)
    if kind == "ln_weight":
        t = 1.0 + 0.1 * s
    elif kind == "bias":
        t = 0.05 * s
    else:
        fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else n
        t = s * (1.5 / math.sqrt(fan_in))
    return t.reshape(shape).to(torch.float32)


def formula_state_dict(shapes):
    """shapes: ordered dict name -> shape (the reference's state_dict).  Bucket
    buffers keep torch.linspace(-20, 20, n) (Agent.py:228, DynamicsPredictors.py:61)."""
    out = {}
    for k, (name, shape) in enumerate(shapes.items()):
        if "buckets" in name:
            out[name] = torch.linspace(-20, 20, shape[0])
            continue
        leaf = name.rsplit(".", 1)[-1]
        is_ln = len(shape) == 1 and name.rsplit(".", 2)[-2].isdigit() and _is_ln(name)
        if leaf == "bias" or leaf.startswith("bias_"):
            kind = "bias"
        elif is_ln:
            kind = "ln_weight"
        else:
            kind = "weight"
        t = formula_tensor(tuple(shape), k, kind)
        if "target_critic" in name:  # target is a deepcopy of the critic (Agent.py:50)
            t = formula_tensor(tuple(shape), list(shapes).index(name.replace("target_critic", "critic")), kind)
        if "mu_head" in name:  # Agent.py:188-189 zero-inits mu_head; keep non-zero for coverage
            t = t * 0.5
        out[name] = t
    return out


_LN_IDX = {"latent_mapper": {"1"}, "logit_net": {"1", "4"}, "logit_generator": {"1", "4"},
           "base_net": {"1", "4"}, "value_net": {"1", "4"}, "upscaler": {"1"}}


def _is_ln(name):
    parts = name.split(".")
    for j, p in enumerate(parts):
        if p in _LN_IDX and j + 1 < len(parts) and parts[j + 1] in _LN_IDX[p]:
            return True
    return False


def replay_data(n, obs_hw, action, seed=0):
    """Synthetic replay contents: u8 frames, U(-1,1) actions,
    N(0,1) rewards, continues 1 except every 1000th (and index 37) = 0."""
    rng = np.random.default_rng(seed)
    frames = rng.integers(0, 256, size=(n, 3, obs_hw[0], obs_hw[1]), dtype=np.uint8)
    acts = rng.uniform(-1, 1, size=(n, action)).astype(np.float32)
    rews = rng.standard_normal(size=(n,)).astype(np.float32)
    conts = np.ones((n,), dtype=np.float32)
    conts[::1000] = 0.0
    if n > 37:
        conts[37] = 0.0
    return frames, acts, rews, conts
