"""WorldModel with the reference's constructor, attributes and methods
(WorldModel.py).  imagine_step / observe_step and the whole training step
(loss, backward, clip_grad_norm_, AdamW: WorldModel.py:148-202) run on
libdreamer_hip; unroll_model keeps a PyTorch-ROCm autograd version for
callers that want the reference's intermediate tensors."""
import os

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from . import hip
from .networks import ContinuePredictor, Decoder, DynamicsPredictor, Encoder, RewardPredictor, SequenceModel
from .utils import symlog, to_twohot  # noqa: F401  (API parity with the reference module)


class WorldModel(nn.Module):
    def __init__(self, hidden_dims, latent_dims, observation_dims, action_dims, training_horizon, batch_size, WM_lr,
                 WM_betas, WM_eps, beta_pred, beta_dyn, beta_rep, num_encoder_filters_1, num_encoder_filters_2,
                 encoder_hidden_layer_nodes, num_decoder_filters_1, num_decoder_filters_2, decoder_hidden_layer_nodes,
                 dyn_pred_hidden_num_nodes_1, dyn_pred_hidden_num_nodes_2, rew_pred_hidden_num_nodes_1,
                 rew_pred_hidden_num_nodes_2, reward_buckets, cont_pred_hidden_num_nodes_1,
                 cont_pred_hidden_num_nodes_2, device="cpu", encoder_depth=4):
        super().__init__()
        self.latent_num_rows, self.latent_num_columns = latent_dims
        self.hidden_dims = hidden_dims
        self.action_dims = action_dims
        self.vector_obs = len(observation_dims) == 1  # BASELINE configs[4] (networks.Encoder)
        self.observation_dim_x, self.observation_dim_y = (observation_dims[0], 1) if self.vector_obs \
            else tuple(observation_dims)
        self.horizon = training_horizon
        self.buckets = reward_buckets
        self.beta_pred, self.beta_dyn, self.beta_rep = beta_pred, beta_dyn, beta_rep
        self.batch_size = batch_size
        R, C = latent_dims
        self.encoder = Encoder(observation_dims, hidden_dims, R, C, num_encoder_filters_1, num_encoder_filters_2,
                               encoder_hidden_layer_nodes, device=device, depth=encoder_depth)
        self.sequence_model = SequenceModel(R, C, hidden_dims, action_dims, num_layers=1, device=device)
        self.dynamics_predictor = DynamicsPredictor(R, C, hidden_dims, dyn_pred_hidden_num_nodes_1,
                                                    dyn_pred_hidden_num_nodes_2, device)
        self.reward_predictor = RewardPredictor(R, C, hidden_dims, rew_pred_hidden_num_nodes_1,
                                                rew_pred_hidden_num_nodes_2, reward_buckets, device=device)
        self.continue_predictor = ContinuePredictor(R, C, hidden_dims, cont_pred_hidden_num_nodes_1,
                                                    cont_pred_hidden_num_nodes_2, device=device)
        self.decoder = Decoder(R, C, observation_dims, hidden_dims, num_decoder_filters_1, num_decoder_filters_2,
                               decoder_hidden_layer_nodes, device=device, depth=encoder_depth)
        self.device = torch.device(device)
        self.optimiser = torch.optim.AdamW(self.parameters(), lr=WM_lr, betas=(WM_betas[0], WM_betas[1]), eps=WM_eps,
                                           weight_decay=1e-6)
        self.scalar = torch.amp.GradScaler(enabled=self.device.type == "cuda")
        self._flat = None
        self._dp = None  # (rank, world, group) under data parallelism
        self.last_losses = None  # device [total, loss_pred, KL_dyn, KL_rep] of the last training_step

    # ---- libdreamer_hip packing ---------------------------------------------
    def dims(self, agent=None):
        d = L.dr_dims()
        self.encoder.fill_dims(d)
        d.action = self.action_dims
        dp, rp, cp = self.dynamics_predictor.logit_net, self.reward_predictor.logit_net, \
            self.continue_predictor.logit_generator
        d.prior_h1, d.prior_h2 = dp[0].out_features, dp[3].out_features
        d.rew_h1, d.rew_h2 = rp[0].out_features, rp[3].out_features
        d.cont_h1, d.cont_h2 = cp[0].out_features, cp[3].out_features
        d.buckets = self.buckets
        self.decoder.fill_dims(d)
        d.precision = 1 if getattr(self, "precision", "fp32") == "bf16" else 0  # DR_PREC_BF16 / DR_PREC_FP32
        # DREAMER_PERSISTENT=0: every entry point as its launch sequence (A/B of the persistent kernels)
        d.launch_form = 1 if os.environ.get("DREAMER_PERSISTENT", "1") == "0" else 0
        if agent is not None:
            if not agent.persistent_ok:
                d.launch_form = 1
            if agent.grad_buffer.is_cuda:
                d.fault = agent.fault_slot().data_ptr()
                d.fault_host = agent.fault_host()[1]
            a, c = agent.actor.base_net, agent.critic.value_net
            d.actor_h1, d.actor_h2 = a[0].out_features, a[3].out_features
            d.critic_h1, d.critic_h2 = c[0].out_features, c[3].out_features
        return d

    def packed(self):
        wm = L.dr_world_model()
        self.encoder.fill(wm)
        g = self.sequence_model.GRU
        wm.w_ih, wm.w_hh, wm.b_ih, wm.b_hh = (L.ptr(t) for t in (g.weight_ih, g.weight_hh, g.bias_ih, g.bias_hh))
        wm.prior = hip.mlp3(self.dynamics_predictor.logit_net)
        wm.reward = hip.mlp3(self.reward_predictor.logit_net)
        wm.cont = hip.mlp3(self.continue_predictor.logit_generator)
        wm.buckets_rew = L.ptr(self.reward_predictor.buckets_rew)
        return wm

    def packed_decoder(self):
        return self.decoder.packed()

    def _grad_structs(self):
        """C structs pointing at the parameters' .grad views (one flat buffer)."""
        e, g = self.encoder, L.dr_world_model()
        for i in range(len(e.feature_extractor) // 2):
            g.conv[i] = hip.linear_grad(e.feature_extractor[2 * i])
        g.map0, g.map1, g.map3 = (hip.linear_grad(e.latent_mapper[j]) for j in (0, 1, 3))
        gru = self.sequence_model.GRU
        g.w_ih, g.w_hh, g.b_ih, g.b_hh = (L.ptr(t.grad) for t in (gru.weight_ih, gru.weight_hh, gru.bias_ih,
                                                                   gru.bias_hh))
        g.prior = hip.mlp3_grad(self.dynamics_predictor.logit_net)
        g.reward = hip.mlp3_grad(self.reward_predictor.logit_net)
        g.cont = hip.mlp3_grad(self.continue_predictor.logit_generator)
        up, ib = self.decoder.upscaler, self.decoder.image_builder
        gd = L.dr_decoder(hip.linear_grad(up[0]), hip.linear_grad(up[1]), hip.linear_grad(up[3]))
        for i in range((len(ib) + 1) // 2):
            gd.convt[i] = hip.linear_grad(ib[2 * i])
        return g, gd

    def _grad_buckets(self, f):
        """Flat-gradient ranges final after each backward stage of
        dr_wm_train_phase (DR_WM_BWD_HEADS, _SCAN, _ENC): the heads and the
        decoder; latent_mapper and the GRU; the encoder convolutions.  They
        are contiguous in the flat buffer (parameter registration order:
        encoder convs, latent_mapper, GRU, heads, decoder)."""
        key = (f.numel, tuple(f.names))
        if getattr(self, "_buckets", (None,))[0] == key:
            return self._buckets[1]
        def stage(n):
            if n.startswith("encoder.feature_extractor."):
                return 2
            if n.startswith("encoder.latent_mapper.") or n.startswith("sequence_model."):
                return 1
            return 0
        lo, hi = [f.numel] * 3, [0] * 3
        for n, p in zip(f.names, f.params):
            k, o = stage(n), f.offsets[n]
            lo[k], hi[k] = min(lo[k], o), max(hi[k], o + -(-p.numel() // 64) * 64)
        for n in f.names:  # each range holds only its own stage's parameters
            o = f.offsets[n]
            for k in range(3):
                if lo[k] <= o < hi[k] and stage(n) != k:
                    raise RuntimeError(f"world-model gradient buckets are not contiguous ({n})")
        out = [(lo[k], hi[k]) if hi[k] > lo[k] else (0, 0) for k in range(3)]
        self._buckets = (key, out)
        return out

    def _ensure_flat(self):
        """Parameters as views of one flat buffer, gradients in another, and
        the optimiser as the fused HIP AdamW over them (same hyper-parameters
        as the reference's torch.optim.AdamW, WorldModel.py:63-69)."""
        from .agent import FlatAdamW, _Flat
        if self._flat is not None and self._flat.intact():
            return self._flat
        g = self.optimiser.param_groups[0]
        self._flat = _Flat(self)
        self.optimiser = FlatAdamW(self._flat, g["lr"], g["betas"], g["eps"], g["weight_decay"])
        return self._flat

    def set_data_parallel(self, rank, world, group=None, force=False):
        """Shard training_step's batch over `world` ranks (one per GPU): the
        mask sum and the loss sums are all-reduced between the step's phases,
        so losses, free-bit clamps and gradients are the global ones, and the
        flat gradient is all-reduced (sum) before clip_grad_norm_.  force=True
        keeps the collective path at world == 1 (tests/test_gpu_rccl.py runs
        it over RCCL on one GPU)."""
        self._dp = (rank, world, group) if (world > 1 or force) else None

    def params_key(self):
        return tuple(p.data_ptr() for p in self.parameters())

    # ---- hot-path steps (HIP) -------------------------------------------------
    def imagine_step(self, hidden_state, latent_state, action):  # WorldModel.py:72-77
        L.require_gpu(hidden_state)
        B = hidden_state.shape[0]
        Hd, Lt = self.hidden_dims, self.latent_num_rows * self.latent_num_columns
        h = hidden_state.reshape(B, Hd).float().contiguous()
        z = latent_state.reshape(B, Lt).float().contiguous()
        a = action.reshape(B, self.action_dims).float().contiguous()
        dev = h.device
        h2, z2 = torch.empty(B, 1, Hd, device=dev), torch.empty(B, 1, self.latent_num_rows, self.latent_num_columns,
                                                               device=dev)
        r, c = torch.empty(B, 1, 1, device=dev), torch.empty(B, 1, 1, device=dev)
        d = self.dims()
        ws = hip.workspace(dev).get("istep", L.query("dr_step_workspace_bytes", d, B))
        L.call("dr_imagine_step", d, self.packed(), B, L.ptr(h), L.ptr(z), L.ptr(a), hip.adhoc(dev).noise(), L.ptr(h2),
               L.ptr(z2), L.ptr(r), L.ptr(c), L.ptr(ws), ws.numel(), hip.stream())
        return h2, z2, r, c

    def observe_step(self, last_latent, last_hidden, last_action, observation):  # WorldModel.py:79-82
        if hip.needs_torch_grad(self.sequence_model, self.encoder):
            return self._observe_step_torch(last_latent, last_hidden, last_action, observation)
        L.require_gpu(observation)
        B = last_hidden.shape[0]
        Hd, Lt = self.hidden_dims, self.latent_num_rows * self.latent_num_columns
        dev = observation.device
        d = self.dims()
        wm = self.packed()
        obs = observation.reshape(B, -1).float().contiguous()
        feat = torch.empty(B, d.enc_hidden, device=dev)
        st = hip.stream()
        ws = hip.workspace(dev).get("enc", L.query("dr_encoder_workspace_bytes", d, B))
        fr = L.dr_frames(None, 0, None, L.ptr(obs), obs.shape[1], 0, 0)
        L.call("dr_encoder_features", d, wm, fr, B, 1, L.ptr(feat), L.ptr(ws), ws.numel(), st)
        z_in = last_latent.reshape(B, Lt).float().contiguous()
        h_in = last_hidden.reshape(B, Hd).float().contiguous()
        a = last_action.reshape(B, self.action_dims).float().contiguous()
        z = torch.empty(B, 1, self.latent_num_rows, self.latent_num_columns, device=dev)
        h = torch.empty(B, 1, Hd, device=dev)
        lg = torch.empty(B, 1, self.latent_num_rows, self.latent_num_columns, device=dev)
        ws2 = hip.workspace(dev).get("obs", L.query("dr_observe_workspace_bytes", d, B))
        L.call("dr_observe_scan", d, wm, B, 1, L.ptr(feat), L.ptr(a), self.action_dims, 0, L.ptr(h_in), L.ptr(z_in),
               hip.adhoc(dev).noise(), L.ptr(z), L.ptr(h), L.ptr(lg), L.ptr(ws2), ws2.numel(), st)
        return z, h, lg

    # ---- world-model training (PyTorch-ROCm this round) ----------------------
    def _sample_torch(self, logits):
        probs = torch.softmax(logits.float(), dim=-1)
        probs = 0.99 * probs + 0.01 * (1.0 / self.latent_num_columns)
        idx = torch.distributions.Categorical(probs=probs).sample()
        return torch.nn.functional.one_hot(idx, self.latent_num_columns).float() + probs - probs.detach()

    def _observe_step_torch(self, last_latent, last_hidden, last_action, observation):
        h = self.sequence_model(last_latent, last_hidden, last_action)
        B, S, _ = h.shape
        logits = self.encoder(h, observation).view(B, S, self.latent_num_rows, self.latent_num_columns)
        return self._sample_torch(logits), h, logits

    def unroll_model(self, observation_sequence_batch, action_sequence_batch, reward_sequence_batch,
                     continue_sequence_batch):  # WorldModel.py:84-146
        B = continue_sequence_batch.shape[0]
        dev = observation_sequence_batch.device
        h = torch.zeros(B, 1, self.hidden_dims, device=dev)
        z = torch.zeros(B, 1, self.latent_num_rows, self.latent_num_columns, device=dev)
        zs, hs, lgs = [], [], []
        for t in range(self.horizon):
            a = action_sequence_batch[:, t - 1:t] if t > 0 else torch.zeros(B, 1, self.action_dims, device=dev)
            z, h, lg = self._observe_step_torch(z, h, a, observation_sequence_batch[:, t:t + 1])
            zs.append(z); hs.append(h); lgs.append(lg)
        post_logits, hid, lat = torch.cat(lgs, 1), torch.cat(hs, 1), torch.cat(zs, 1)
        prior_logits = self.dynamics_predictor(hid)
        dec_mu = self.decoder(hid, lat)
        reward_logits = self.reward_predictor(hid[:, 1:], lat[:, 1:])
        _, cont_logits = self.continue_predictor(hid[:, 1:], lat[:, 1:])
        obs_t = observation_sequence_batch[:, :self.horizon]
        rew_t = reward_sequence_batch[:, :self.horizon - 1]
        cont_t = continue_sequence_batch[:, :self.horizon - 1]
        obs_ll = -(dec_mu.float() - obs_t.float()).pow(2).sum(dim=[-1] if self.vector_obs else [-3, -2, -1])
        cont_ll = torch.nn.functional.binary_cross_entropy_with_logits(cont_logits, cont_t, reduction="none")
        rew_ll = torch.sum(to_twohot(rew_t, self.reward_predictor.buckets_rew)
                           * torch.nn.functional.log_softmax(reward_logits, dim=-1), dim=-1, keepdim=True)
        return prior_logits[:, 1:], post_logits[:, 1:], obs_ll[:, 1:], rew_ll, cont_ll

    def training_step(self, observation_sequences, action_sequences, reward_sequences, continue_sequences):
        """WorldModel.training_step (WorldModel.py:148-202) on libdreamer_hip:
        posterior scan, heads, decoder, losses and the full backward in one
        launch sequence (dr_wm_train_grads), then clip_grad_norm_(100) and
        AdamW fused over the flat parameter buffer.  fp32 throughout: the
        reference's fp16 autocast + GradScaler reduce, in fp32, to the plain
        backward plus a skipped step when the loss or a gradient is non-finite
        (the reference prints and returns before its backward, 191-193).
        Returns the total loss as a 0-d device tensor."""
        return self.train_step_hip(observation_sequences, action_sequences, reward_sequences, continue_sequences)

    def train_step_hip(self, obs, act, rew, cont, noise_q=None, outputs=None, step=True):
        """obs (B,S,3,H,W) holding 0..255 (Buffer.sample_sequences), act
        (B,S,A), rew / cont (B,S,1).  noise_q: explicit Exp(1) draws
        (T, B*rows, cols) for the posterior samples (parity tests), else
        Philox.  outputs: optional dict that receives the time-major posterior
        hiddens / latents / logits.  step=False leaves the parameters alone
        (gradients only)."""
        L.require_gpu(obs)
        B, S = act.shape[:2]
        Hh, Ww, A = self.observation_dim_x, self.observation_dim_y, self.action_dims
        obs = obs.float().contiguous()
        act = act.float().contiguous()
        rew = rew.float().reshape(B, S).contiguous()
        cont = cont.float().reshape(B, S).contiguous()
        if self.vector_obs:  # (B, S, D) f32 observations, used as given
            fr = L.dr_frames(None, 0, None, L.ptr(obs), S * Hh, Hh, 0, 0)
        else:
            fr = L.dr_frames(None, 0, None, L.ptr(obs), S * 3 * Hh * Ww, 3 * Hh * Ww, 1, 0)
        bt = L.dr_wm_batch(L.ptr(act), S * A, A, L.ptr(rew), L.ptr(cont), S, 1)
        return self._train(fr, bt, B, S, obs.device, noise_q, outputs, step)

    def train_step_ring(self, buffer, starts, noise_q=None, outputs=None, step=True):
        """The same step fed straight from the device replay ring: frames are
        read as u8 by the first conv's loader, actions / rewards / continues
        gathered for the first `horizon` steps of each window (no float32
        observation tensor is materialised, Buffer.py:58-61)."""
        dev = buffer.device
        B, T = len(starts), self.horizon
        st = torch.as_tensor(np.asarray(starts), dtype=torch.int64).to(dev, non_blocking=True) \
            if not isinstance(starts, torch.Tensor) else starts
        win = self._win.get((B, T)) if hasattr(self, "_win") else None
        if win is None:
            self._win = getattr(self, "_win", {})
            win = self._win[(B, T)] = (torch.empty(B, T, self.action_dims, device=dev), torch.empty(B, T, device=dev),
                                       torch.empty(B, T, device=dev))
        act, rew, cont = win
        m = buffer._mirror()
        L.call("dr_replay_gather", buffer.capacity, B, T, 0, self.action_dims, None, L.ptr(m["actions"]),
               L.ptr(m["rewards"]), L.ptr(m["continues"]), L.ptr(st), None, L.ptr(act), L.ptr(rew), L.ptr(cont),
               hip.stream())
        fr = buffer.frames_struct(st)
        bt = L.dr_wm_batch(L.ptr(act), T * self.action_dims, self.action_dims, L.ptr(rew), L.ptr(cont), T, 1)
        return self._train(fr, bt, B, T, dev, noise_q, outputs, step)

    def _train(self, fr, bt, B, S, dev, noise_q, outputs, step):
        T = self.horizon
        if S < T or T < 2:
            raise ValueError(f"training_step needs sequences of at least horizon={T} >= 2 steps (got {S})")
        Hd, R, C = self.hidden_dims, self.latent_num_rows, self.latent_num_columns
        f = self._ensure_flat()
        d = self.dims()
        row0 = 0 if self._dp is None else self._dp[0] * B  # Philox keyed by the global row
        noise = hip.explicit_noise(q=noise_q, device=dev) if noise_q is not None else hip.adhoc(dev).noise(row0=row0)
        cfg = L.dr_wm_loss_cfg(self.beta_pred, self.beta_dyn, self.beta_rep)
        if getattr(self, "_scratch", None) is None or self._scratch[0].device != torch.device(dev):
            self._scratch = (torch.empty(4, device=dev), torch.zeros(1, dtype=torch.int32, device=dev),
                             torch.zeros(1, device=dev), torch.empty(512, device=dev), torch.zeros(8, device=dev))
        losses, skip, sq, sq_part, stats = self._scratch
        hid = lat = plog = None
        if outputs is not None:
            hid = torch.empty(T, B, Hd, device=dev)
            lat = torch.empty(T, B, R, C, device=dev)
            plog = torch.empty(T, B, R, C, device=dev)
        gw, gd = self._grad_structs()
        ws = hip.workspace(dev).get("wm_train", L.query("dr_wm_train_workspace_bytes", d, B, T))
        st = hip.stream()
        args = (d, self.packed(), self.packed_decoder(), B, T, fr, bt)
        tail = (L.ptr(losses), L.ptr(skip), gw, gd, L.ptr(hid), L.ptr(lat), L.ptr(plog), L.ptr(ws), ws.numel(), st)
        if self._dp is None:
            L.call("dr_wm_train_phase", *args, noise, cfg, 7, L.ptr(stats), 0, *tail)
        else:
            import torch.distributed as dist
            rank, world, group = self._dp
            rows = world * B * (T - 1)
            L.call("dr_wm_train_phase", *args, noise, cfg, 1, L.ptr(stats), rows, *tail)
            dist.all_reduce(stats[0:1], group=group)
            L.call("dr_wm_train_phase", *args, noise, cfg, 2, L.ptr(stats), rows, *tail)
            dist.all_reduce(stats[1:5], group=group)
            # backward in three stages, each gradient bucket all-reduced (on
            # the communicator's stream) while the next stage computes
            works = []
            for bit, (lo, hi) in zip((8, 16, 32), self._grad_buckets(f)):
                L.call("dr_wm_train_phase", *args, noise, cfg, bit, L.ptr(stats), rows, *tail)
                if hi > lo:
                    works.append(dist.all_reduce(f.grad[lo:hi], group=group, async_op=True))
            for w in works:
                w.wait()
        if outputs is not None:
            outputs.update(hiddens=hid, latents=lat, post_logits=plog)
        if step:
            # GradScaler semantics: no update when the loss or a gradient is non-finite
            L.call("dr_nonfinite", f.numel, f.grad.data_ptr(), skip.data_ptr(), st)
            sq.zero_()
            L.call("dr_sqnorm_multi", f.numel, f.grad.data_ptr(), sq.data_ptr(), sq_part.data_ptr(), st)
            self.optimiser.fused_step(sqnorm=sq, max_norm=100.0, skip=skip)
        self.last_losses, self.last_skip, self.last_sqnorm = losses, skip, sq
        return losses[0].clone()
