"""Dreamer: the reference's top-level agent (Dreamer.py) on the MI355X engine.

Same constructor (config dict + device), attributes, methods and state_dict
layout, so train_car_racer.py runs unchanged.  train_Agent -- the metric's
unit of work -- runs as one fused device-resident epoch (engine.py); the
world-model step stays PyTorch-ROCm this round."""
import os

import numpy as np
import torch
import torch.nn as nn
from tqdm import tqdm

from . import _lib as L
from . import hip
from .agent import Agent
from .buffer import Buffer
from .utils import _sanitize_for_save
from .world_model import WorldModel


class _DreamFn(torch.autograd.Function):
    """dream_episodes as one autograd node: forward = dr_imagine_fwd, backward
    = dr_imagine_bwd (BPTT through the unroll into the actor's parameters).
    The world model receives no gradient (the reference's WM grads from this
    path are discarded, WorldModel.py:195)."""

    @staticmethod
    def forward(ctx, dreamer, z0, h0, *actor_params):
        ctx.set_materialize_grads(False)
        out, tape = dreamer._imagine_raw(z0, h0)
        ctx.dreamer, ctx.tape = dreamer, tape
        ctx.save_for_backward(out[0], out[1], out[2])
        return out

    @staticmethod
    def backward(ctx, g_lat, g_hid, g_act, g_rew, g_cont, g_mu, g_sig):
        for g, n in ((g_rew, "rewards"), (g_cont, "continues")):
            if g is not None and bool(torch.any(g != 0)):
                raise NotImplementedError(f"gradient through imagined {n} is not part of the reference's loss")
        lat, hid, act = ctx.saved_tensors
        dr = ctx.dreamer
        ag = dr.agent
        grad_flat = torch.zeros_like(ag.fa.flat)
        f = ag.fa
        gptr = lambda n: grad_flat.data_ptr() + 4 * f.offsets[n]
        gs = L.dr_actor(*(L.dr_linear(gptr(w), gptr(b)) for w, b in (
            ("base_net.0.weight", "base_net.0.bias"), ("base_net.1.weight", "base_net.1.bias"),
            ("base_net.3.weight", "base_net.3.bias"), ("base_net.4.weight", "base_net.4.bias"),
            ("mu_head.weight", "mu_head.bias"), ("log_sig_head.weight", "log_sig_head.bias"))))
        B, H1 = hid.shape[:2]
        d = dr.world_model.dims(ag)
        c = lambda t: None if t is None else t.float().contiguous()
        g_mu, g_sig, g_act, g_lat, g_hid = (c(t) for t in (g_mu, g_sig, g_act, g_lat, g_hid))
        ws = hip.workspace(hid.device).get("im_bwd", L.query("dr_imagine_workspace_bytes", d, B, H1 - 1))
        L.call("dr_imagine_bwd", d, dr.world_model.packed(), ag.actor_struct(), B, H1 - 1, L.ptr(lat), L.ptr(hid),
               L.ptr(act), L.ptr(g_mu), L.ptr(g_sig), L.ptr(g_act), L.ptr(g_lat), L.ptr(g_hid), L.ptr(ctx.tape), gs,
               L.ptr(ws), ws.numel(), hip.stream())
        grads = [grad_flat[f.offsets[n]:f.offsets[n] + p.numel()].view_as(p) for n, p in zip(f.names, f.params)]
        return (None, None, None, *grads)


class Dreamer(nn.Module):
    def __init__(self, config, device):
        super().__init__()
        c = config
        self.hidden_state_dims = c["hidden_state_dims"]
        self.action_dims = c["action_dims"]
        self.observation_dims = tuple(c["observation_dims"])
        self.latent_state_dims = tuple(c["latent_state_dims"])
        device = torch.device(device)
        self.world_model = WorldModel(
            c["hidden_state_dims"], tuple(c["latent_state_dims"]), tuple(c["observation_dims"]), c["action_dims"],
            c["horizon"], c["batch_size"], c["world_model_lr"], tuple(c["world_model_betas"]), c["world_model_eps"],
            c["beta_prediction"], c["beta_dynamics"], c["beta_representation"], c["encoder_filter_num_1"],
            c["encoder_filter_num_2"], c["encoder_hidden_layer_nodes"], c["decoder_filter_num_1"],
            c["decoder_filter_num_2"], c["decoder_hidden_layer_nodes"], c["dyn_pred_hidden_num_nodes_1"],
            c["dyn_pred_hidden_num_nodes_2"], c["rew_pred_hidden_num_nodes_1"], c["rew_pred_hidden_num_nodes_2"],
            c["critic_reward_buckets"], c["cont_pred_hidden_num_nodes_1"], c["cont_pred_hidden_num_nodes_2"],
            device=device, encoder_depth=int(c.get("encoder_depth", 4)))
        self.agent = Agent(
            c["action_dims"], tuple(c["latent_state_dims"]), c["hidden_state_dims"], c["hidden_layer_actor_1_size"],
            c["hidden_layer_actor_2_size"], c["hidden_layer_critic_1_size"], c["hidden_layer_critic_2_size"],
            c["critic_reward_buckets"], c["actor_lr"], tuple(c["actor_betas"]), c["actor_eps"], c["critic_lr"],
            tuple(c["critic_betas"]), c["critic_eps"], c["nu"], c["lambda_"], c["gamma"], device=device)
        self.buffer = Buffer(c["buffer_size"], c["sequence_length"], c["action_dims"], tuple(c["observation_dims"]),
                             device=device)
        self.horizon = c["horizon"]
        self.batch_size = c["batch_size"]
        self.sequence_length = c["sequence_length"]
        self.training_iterations = c["training_iterations"]
        self.random_iterations = c["random_iterations"]
        self.WM_epochs = c["WM_epochs"]
        self.AC_epochs = c["AC_epochs"]
        self.seed = c["seed"]
        # extra config key: "fp32" parity mode (default) or "bf16" perf mode
        self.precision = c.get("precision", "fp32")
        # on by default from round 4: bit-equal to sequential epochs
        # (test_pipelined_epochs_match_sequential), 1.04x at AC_epochs = 2 and
        # 1.16x at 10; pipeline_epochs: false restores
        # the sequential loop
        self.pipeline_epochs = bool(c.get("pipeline_epochs", True))
        self.world_model.precision = self.precision  # encoder kernels: bf16 MFMA in perf mode
        if self.precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {self.precision!r}")
        self.device = device
        self.agent_obs = None
        self.agent_hidden = None
        self.agent_latent = None
        self._engine = None
        self.world = None  # (rank, size, group) for data-parallel train_Agent

    # ------------------------------------------------------------- imagination
    def _imagine_raw(self, z0, h0, eps=None, q=None):
        L.require_gpu(h0)
        B = h0.shape[0]
        H = self.horizon
        R, C = self.latent_state_dims
        A = self.action_dims
        dev = h0.device
        d = self.world_model.dims(self.agent)
        lat = torch.empty(B, H + 1, R, C, device=dev)
        hid = torch.empty(B, H + 1, self.hidden_state_dims, device=dev)
        act, mu, sg = (torch.empty(B, H, A, device=dev) for _ in range(3))
        rew, cont = torch.empty(B, H, 1, device=dev), torch.empty(B, H, 1, device=dev)
        tape = torch.empty(L.query("dr_imagine_tape_bytes", d, B, H), dtype=torch.uint8, device=dev)
        ws = hip.workspace(dev).get("im", L.query("dr_imagine_workspace_bytes", d, B, H))
        if eps is None and q is None:
            nz = hip.adhoc(dev).noise()
        else:
            nz = hip.explicit_noise(q=q, eps=eps, device=dev)
        z = z0.reshape(B, -1).float().contiguous()
        h = h0.reshape(B, -1).float().contiguous()
        L.call("dr_imagine_fwd", d, self.world_model.packed(), self.agent.actor_struct(), B, H, L.ptr(z), L.ptr(h),
               nz, 0, L.ptr(lat), L.ptr(hid), L.ptr(act), L.ptr(rew), L.ptr(cont), L.ptr(mu), L.ptr(sg), L.ptr(tape),
               L.ptr(ws), ws.numel(), hip.stream())
        return (lat, hid, act, rew, cont, mu, sg), tape

    def dream_episodes(self, starting_latent_state_batch, starting_hidden_state_batch):
        """Dreamer.dream_episodes (Dreamer.py:143-175) as one HIP unroll."""
        self.agent._ensure_flat()
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.agent.actor.parameters()):
            return _DreamFn.apply(self, starting_latent_state_batch.detach(), starting_hidden_state_batch.detach(),
                                  *self.agent.fa.params)
        return self._imagine_raw(starting_latent_state_batch, starting_hidden_state_batch)[0]

    def warm_start_generator(self, observation_seq_batch, action_seq_batch, sequence_length):
        """Dreamer.warm_start_generator (Dreamer.py:244-262): time-batched conv
        encoder over the S/2 warm-up frames, then the posterior scan."""
        obs = observation_seq_batch.float().contiguous()
        L.require_gpu(obs)
        B, S = obs.shape[:2]
        T = sequence_length // 2
        d = self.world_model.dims(self.agent)
        wm = self.world_model.packed()
        dev = obs.device
        fe = int(np.prod(obs.shape[2:]))
        fr = L.dr_frames(None, 0, None, L.ptr(obs), S * fe, fe, 1)
        feat = torch.empty(T * B, d.enc_hidden, device=dev)
        st = hip.stream()
        ws = hip.workspace(dev).get("enc", L.query("dr_encoder_workspace_bytes", d, T * B))
        L.call("dr_encoder_features", d, wm, fr, B, T, L.ptr(feat), L.ptr(ws), ws.numel(), st)
        act = action_seq_batch.float().contiguous()
        A = act.shape[-1]
        R, C = self.latent_state_dims
        z = torch.empty(B, 1, R, C, device=dev)
        h = torch.empty(B, 1, self.hidden_state_dims, device=dev)
        ws2 = hip.workspace(dev).get("obs", L.query("dr_observe_workspace_bytes", d, B))
        L.call("dr_observe_scan", d, wm, B, T, L.ptr(feat), L.ptr(act), act.shape[1] * A, A, None, None,
               hip.adhoc(dev).noise(), L.ptr(z), L.ptr(h), None, L.ptr(ws2), ws2.numel(), st)
        return z, h

    # --------------------------------------------------------------- training
    @property
    def engine(self):
        if self._engine is None:
            from .engine import ImaginationEngine
            self._engine = ImaginationEngine(self, world=self.world)
        return self._engine

    def train_Agent(self):
        """Dreamer.train_Agent (Dreamer.py:264-287): AC_epochs fused epochs."""
        if self.AC_epochs > 1 and self.pipeline_epochs and not self.engine.persistent_chain():
            # config key pipeline_epochs (default on): the epochs' window
            # starts are drawn up front (same np.random order); the warm start
            # of epoch e+1 then overlaps epoch e's update (engine.run_many),
            # bit for bit the sequential launch-form epochs.  Where the chain
            # runs as the persistent kernels (B <= 128 per GPU) the sequential
            # epochs below are faster (a persistent kernel needs every CU, so
            # it cannot share the chip with an overlapped warm start; measured
            # in bench.py's configs1_B64_ac_epochs2)
            B = self.batch_size if self.world is None else self.engine.B
            starts = [self.buffer.sample_start_indices(B) for _ in range(self.AC_epochs)]
            losses = self.engine.run_many(starts)
            return losses[:, 0].mean(dim=0), losses[:, 1].mean(dim=0)
        if self.AC_epochs == 1:
            # one epoch: one copy of the two loss slots (the loop below costs
            # clone + cat + mean per loss, six small launches outside the
            # captured graphs, each behind a dispatch gap); the mean of one
            # value is that value, bit for bit
            starts = self.buffer.sample_start_indices(self.batch_size if self.world is None else self.engine.B)
            self.engine.run(starts)
            losses = self.agent.loss_buffer[0:2].clone()
            return losses[0], losses[1]
        la, lc = [], []
        for _ in tqdm(range(self.AC_epochs), desc="Training Agent in Dreams", leave=False):
            starts = self.buffer.sample_start_indices(self.batch_size if self.world is None else self.engine.B)
            a, c = self.engine.run(starts)
            la.append(a.clone())
            lc.append(c.clone())
        return torch.cat(la).mean(dim=0), torch.cat(lc).mean(dim=0)

    def train_world_model(self):  # Dreamer.py:228-242
        out = []
        for _ in tqdm(range(self.WM_epochs), desc="Training World Model On Buffer Data", leave=False):
            if self.device.type == "cuda":
                # same np.random draws as sample_sequences; frames stay u8 in HBM
                starts = self.buffer.sample_start_indices(self.batch_size)
                out.append(self.world_model.train_step_ring(self.buffer, starts))
            else:
                obs, act, rew, cont, _ = self.buffer.sample_sequences(batch_size=self.batch_size)
                out.append(self.world_model.training_step(obs, act, rew, cont))
        return out

    def load_pretrained_dreamer(self, path):
        self.load_state_dict(torch.load(path, weights_only=True))

    def save_trained_Dreamer(self, save_path):
        torch.save(self.state_dict(), save_path)

    # ---- true resume (beyond the reference, whose checkpoints are weights only:
    # Dreamer.py:289-293, 347-354).  One torch.save file of tensors and plain
    # scalars (loads with weights_only=True): the reference-layout state_dict,
    # the three AdamW states (moments + step), S, the engine / ad-hoc Philox
    # states, numpy's and torch's CPU generators (window sampling), the replay
    # ring and the env seed counter.  Resuming reproduces the uninterrupted
    # run's TRAINING UPDATES (train_world_model / train_Agent) bit for bit
    # (tests/test_gpu_api.py::test_training_state_resume).  The in-progress env
    # episode is not part of the state (the env object, agent_obs / hidden /
    # latent): after a resume rollout_policy starts a fresh episode with
    # env.reset(seed), so runs that resume mid-episode diverge from there.
    TRAINING_STATE_FORMAT = "dreamer_amd.training_state.v1"

    def training_state(self):
        ag, wm, buf = self.agent, self.world_model, self.buffer
        ag._ensure_flat()
        wm._ensure_flat()
        cpu = lambda t: t.detach().cpu().clone()
        opt = lambda o: {"exp_avg": cpu(o.exp_avg), "exp_avg_sq": cpu(o.exp_avg_sq), "step": cpu(o.step_dev)}
        name, keys, pos, has_gauss, gauss = np.random.get_state()
        er, ar = hip.rng(self.device), hip.adhoc(self.device)
        return {
            "format": self.TRAINING_STATE_FORMAT,
            "model": {k: cpu(v) for k, v in self.state_dict().items()},
            "opt_actor": opt(ag.actor_optimiser), "opt_critic": opt(ag.critic_optimiser), "opt_wm": opt(wm.optimiser),
            "S": cpu(ag.S_dev),
            "rng_engine": cpu(er.state), "rng_engine_counter": int(er.counter),
            "rng_adhoc": cpu(ar.state), "rng_adhoc_counter": int(ar.counter),
            "np_rng": {"keys": torch.from_numpy(np.asarray(keys, dtype=np.int64)), "pos": int(pos),
                       "has_gauss": int(has_gauss), "gauss": float(gauss)},
            "torch_rng": torch.get_rng_state(),
            "buffer": {"obs": torch.from_numpy(buf.observation_buffer.copy()),
                       "act": torch.from_numpy(buf.action_buffer.copy()),
                       "rew": torch.from_numpy(buf.reward_buffer.copy()),
                       "cont": torch.from_numpy(buf.continue_buffer.copy()),
                       "next_idx": int(buf.next_idx), "size": int(buf.size)},
            "seed": int(self.seed),
        }

    def save_training_state(self, path):
        torch.save(self.training_state(), path)

    def load_training_state(self, path_or_state):
        st = path_or_state if isinstance(path_or_state, dict) else torch.load(path_or_state, weights_only=True)
        if st.get("format") != self.TRAINING_STATE_FORMAT:
            raise ValueError(f"not a {self.TRAINING_STATE_FORMAT} file: {st.get('format')!r}")
        self.load_state_dict({k: v.to(self.device) for k, v in st["model"].items()})
        ag, wm, buf = self.agent, self.world_model, self.buffer
        ag._ensure_flat()
        wm._ensure_flat()
        for o, k in ((ag.actor_optimiser, "opt_actor"), (ag.critic_optimiser, "opt_critic"), (wm.optimiser, "opt_wm")):
            o.exp_avg.copy_(st[k]["exp_avg"])
            o.exp_avg_sq.copy_(st[k]["exp_avg_sq"])
            o.step_dev.copy_(st[k]["step"])
        ag.S_dev.copy_(st["S"])
        er, ar = hip.rng(self.device), hip.adhoc(self.device)
        er.state.copy_(st["rng_engine"])
        er.counter = int(st["rng_engine_counter"])
        ar.state.copy_(st["rng_adhoc"])
        ar.counter = int(st["rng_adhoc_counter"])
        r = st["np_rng"]
        np.random.set_state(("MT19937", r["keys"].numpy().astype(np.uint32), int(r["pos"]), int(r["has_gauss"]),
                             float(r["gauss"])))
        torch.set_rng_state(st["torch_rng"])
        b = st["buffer"]
        buf.observation_buffer[...] = b["obs"].numpy()
        buf.action_buffer[...] = b["act"].numpy()
        buf.reward_buffer[...] = b["rew"].numpy()
        buf.continue_buffer[...] = b["cont"].numpy()
        buf.next_idx, buf.size = int(b["next_idx"]), int(b["size"])
        buf._dirty = list(range(buf.capacity))  # the device mirror re-uploads on next use
        self.seed = int(st["seed"])

    # ------------------------------------------------- acting (batch-1, HIP)
    def _obs_tensor(self, observation):
        obs = observation.transpose(2, 0, 1).astype(np.uint8)
        norm = (obs.astype(np.float32) / 255.0) - 0.5
        return norm, torch.tensor(norm, dtype=torch.float32, device=self.device).unsqueeze(0).unsqueeze(0)

    def act_step(self, observation, z=None, h=None, a=None, deterministic=False):
        """One env step of the acting loop in ONE launch (dr_act_step): with
        (z, h, a) from the previous step, h' = GRU(z, h, a) (observe_step,
        WorldModel.py:79-82); without them, h' = 0 (episode start,
        Dreamer.py:186-187).  Then z' = Encoder.encode(h', observation) and
        a' = Actor.act(h', z', deterministic).  observation: the env's H x W x 3
        uint8 frame.  Returns (a', mu, sigma, z', h') shaped (1, 1, ...)."""
        dev = self.device
        L.require_gpu(torch.empty(0, device=dev))
        if self.world_model.vector_obs or getattr(self, "_act_unfused", False):
            return self._act_step_unfused(observation, z, h, a, deterministic)
        d = self.world_model.dims(self.agent)
        self.agent._ensure_flat()
        R, C = self.latent_state_dims
        A, Hd = self.action_dims, self.hidden_state_dims
        st = getattr(self, "_act_bufs", None)
        if st is None:
            H_, W_ = self.observation_dims
            st = self._act_bufs = dict(
                pin=torch.empty(H_, W_, 3, dtype=torch.uint8).pin_memory(),
                frame=torch.empty(H_, W_, 3, dtype=torch.uint8, device=dev),
                h0=torch.zeros(Hd, device=dev),
                status=torch.zeros(1, dtype=torch.int32, device=dev),
                status_host=torch.zeros(1, dtype=torch.int32).pin_memory(),
                ws=torch.empty(L.query("dr_act_step_workspace_bytes", d), dtype=torch.uint8, device=dev))
        self._act_sync()  # the previous step's copy out of the pinned staging buffer has run (and it was ok)
        st["pin"].numpy()[...] = observation
        st["frame"].copy_(st["pin"], non_blocking=True)
        has_prev = z is not None
        zp = z.reshape(-1).float().contiguous() if has_prev else None
        hp = h.reshape(-1).float().contiguous() if has_prev else st["h0"]
        ap = a.reshape(-1).float().contiguous() if has_prev else None
        z2 = torch.empty(1, 1, R, C, device=dev)
        h2 = torch.empty(1, 1, Hd, device=dev)
        a2, mu, sg = (torch.empty(1, 1, A, device=dev) for _ in range(3))
        try:
            L.call("dr_act_step", d, self.world_model.packed(), self.agent.actor_struct(), L.ptr(st["frame"]),
                   int(has_prev), L.ptr(zp), L.ptr(hp), L.ptr(ap), hip.adhoc(dev).noise(), int(deterministic),
                   L.ptr(z2), L.ptr(h2), L.ptr(a2), L.ptr(mu), L.ptr(sg), None, L.ptr(st["status"]),
                   L.ptr(st["ws"]), st["ws"].numel(), hip.stream())
        except L.HipError as e:
            if e.code != L.DR_E_UNSUPPORTED:
                raise
            # the device cannot hold the one-launch grid, or the widths are not the ones the
            # kernel's register batches are sized for (e.g. the 5-layer VAE): the unfused launches
            self._act_unfused = True
            return self._act_step_unfused(observation, z, h, a, deterministic)
        # the status word travels back with the step (4 bytes behind the kernel);
        # _act_sync / act_check raise on a timed-out grid barrier
        st["status_host"].copy_(st["status"], non_blocking=True)
        self._act_ev = torch.cuda.Event()
        self._act_ev.record()
        return a2, mu, sg, z2, h2

    def act_check(self):
        """Wait for the last act_step and raise if its one-launch kernel hit a
        grid-barrier timeout (its outputs are then NaN, never a state)."""
        self._act_sync()

    def _act_step_unfused(self, observation, z, h, a, deterministic):
        """The same step through the unfused HIP launches -- dr_gru_cell,
        dr_encoder_features + dr_observe_scan (Encoder.encode), dr_actor_act:
        vector observations (BASELINE configs[4]) and devices that cannot hold
        dr_act_step's grid co-resident."""
        dev = self.device
        wm = self.world_model
        if wm.vector_obs:
            obs = torch.as_tensor(np.asarray(observation, dtype=np.float32), device=dev).view(1, 1, -1)
        else:
            _, obs = self._obs_tensor(observation)
        if z is None:
            h2 = torch.zeros(1, 1, self.hidden_state_dims, device=dev)
        else:
            h2 = wm.sequence_model(z.reshape(1, 1, -1), h.reshape(1, 1, -1), a.reshape(1, 1, -1))
        z2, _ = wm.encoder.encode(h2, obs)
        a2, mu, sg = self.agent.actor.act(h2, z2, deterministic=deterministic)
        return a2, mu, sg, z2, h2

    def _agent_obs(self, observation):
        """The env observation as the agent keeps it (Dreamer.py:181-183): a
        normalised CHW frame, or the raw f32 vector."""
        if self.world_model.vector_obs:
            return np.asarray(observation, dtype=np.float32)
        return (observation.transpose(2, 0, 1).astype(np.float32) / 255.0) - 0.5

    def _buffer_obs(self, agent_obs):
        if self.world_model.vector_obs:
            return agent_obs
        return ((agent_obs + 0.5) * 255.0).astype(np.uint8)

    def _act_sync(self):
        ev = getattr(self, "_act_ev", None)
        if ev is None:
            return
        ev.synchronize()
        st = self._act_bufs
        if int(st["status_host"][0]) != 0:
            st["status"].zero_()
            st["status_host"].zero_()
            self._act_ev = None
            raise RuntimeError("dr_act_step: a grid barrier timed out (the acting grid was not co-resident, e.g. "
                               "beside a long-running kernel); that step's outputs are NaN")

    def rollout_policy(self, env, random_policy=False):  # Dreamer.py:177-226
        """Same env / buffer sequence as the reference; the device work of each
        env step (observe_step + the next step's act) is one dr_act_step launch."""
        with torch.no_grad():
            if self.agent_obs is None:
                observation, _ = env.reset(seed=self.seed)
                self.agent_obs = self._agent_obs(observation)
                _, _, _, self.agent_latent, self.agent_hidden = self.act_step(observation)
            action = None
            if not random_policy:  # the current actor's action for the current state
                action, _, _ = self.agent.actor.act(self.agent_hidden, self.agent_latent, deterministic=False)
            for _ in range(self.sequence_length):
                if random_policy:
                    action_np = env.action_space.sample()
                    action = torch.tensor(action_np, dtype=torch.float32, device=self.device).view(1, 1, -1)
                else:
                    action_np = action.detach().cpu().numpy().reshape(-1)
                    self.act_check()
                observation_, reward, terminated, truncated, _ = env.step(action_np)
                done = terminated or truncated
                self.buffer.add_to_buffer(self._buffer_obs(self.agent_obs), action_np, reward, 1 - done)
                if done:
                    self.seed += 1
                    observation, _ = env.reset(seed=self.seed)
                    self.agent_obs = self._agent_obs(observation)
                    action, _, _, self.agent_latent, self.agent_hidden = self.act_step(observation)
                else:
                    self.agent_obs = self._agent_obs(observation_)
                    action, _, _, self.agent_latent, self.agent_hidden = self.act_step(
                        observation_, self.agent_latent, self.agent_hidden, action)

    def evaluate_agent(self, env, eval_episodes):  # Dreamer.py:295-322
        rewards = []
        with torch.no_grad():
            for _ in tqdm(range(eval_episodes), desc="Evaluating Agent", leave=False):
                self.seed += 1
                total = 0
                observation, _ = env.reset(seed=self.seed)
                action, _, _, latent, hidden = self.act_step(observation, deterministic=True)
                done = False
                while not done:
                    action_np = action.detach().cpu().numpy().squeeze(0).squeeze(0)
                    self.act_check()
                    observation_, reward, terminated, truncated, _ = env.step(action_np)
                    total += reward
                    done = terminated or truncated
                    if not done:
                        action, _, _, latent, hidden = self.act_step(observation_, latent, hidden, action,
                                                                     deterministic=True)
                rewards.append(total)
        return torch.tensor(rewards, dtype=torch.float32, device=self.device).mean()

    def train_dreamer(self, env, eval_env):  # Dreamer.py:324-372
        WM_loss_list, actor_loss_list, critic_loss_list, evaluation_list = [], [], [], []
        print("Starting Training...")
        print("Starting Random Kickstart.")
        for _ in tqdm(range(self.random_iterations), desc="Kickstarting Dreamer Agent.", leave=True):
            self.rollout_policy(env, random_policy=True)
            WM_loss_list.append([x.detach().cpu().item() for x in self.train_world_model()])
        print("Starting Training Loop...")
        evaluation_list.append(self.evaluate_agent(eval_env, eval_episodes=3).detach().cpu().item())
        for it in tqdm(range(self.training_iterations), desc="Training Dreamer Agent.", leave=True):
            self.rollout_policy(env, random_policy=False)
            wm_loss = self.train_world_model()
            actor_loss, critic_loss = self.train_Agent()
            WM_loss_list.append([x.detach().cpu().item() for x in wm_loss])
            actor_loss_list.append(actor_loss.detach().cpu().item())
            critic_loss_list.append(critic_loss.detach().cpu().item())
            if it % 1000 == 0:
                os.makedirs("./models", exist_ok=True)
                self.save_trained_Dreamer(os.path.join("./models", f"agent_checkpoint_{it}.pth"))
                self.save_trained_Dreamer(os.path.join("./models", "agent_latest.pth"))
                np.savez(os.path.join("./models", "training_logs.npz"),
                         world_model_loss=_sanitize_for_save(WM_loss_list),
                         actor_loss=_sanitize_for_save(actor_loss_list),
                         critic_loss=_sanitize_for_save(critic_loss_list),
                         rewards=_sanitize_for_save(evaluation_list))
            if it % 500 == 0:
                evaluation_list.append(self.evaluate_agent(eval_env, eval_episodes=3).detach().cpu().item())
        print("Training Complete.")
        evaluation_list.append(self.evaluate_agent(eval_env, eval_episodes=10).detach().cpu().item())
        return WM_loss_list, actor_loss_list, critic_loss_list, evaluation_list

    def Run(self, env, env_seed, render=True):  # Dreamer.py:374-401
        total = 0
        observation, _ = env.reset(seed=env_seed)
        with torch.no_grad():
            action, _, _, latent, hidden = self.act_step(observation, deterministic=True)
        done = False
        while not done:
            if render:
                env.render()
            action_np = action.detach().cpu().numpy().squeeze(0).squeeze(0)
            self.act_check()
            observation_, reward, terminated, truncated, _ = env.step(action_np)
            total += reward
            done = terminated or truncated
            if not done:
                with torch.no_grad():
                    action, _, _, latent, hidden = self.act_step(observation_, latent, hidden, action,
                                                                 deterministic=True)
        return total
