"""WorldModel with the reference's constructor, attributes and methods
(WorldModel.py).  imagine_step / observe_step run on libdreamer_hip; the
training step (SURVEY §8f "next") runs its unroll with the modules' own
PyTorch-ROCm forward so gradients reach every world-model weight."""
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
                 cont_pred_hidden_num_nodes_2, device="cpu"):
        super().__init__()
        self.latent_num_rows, self.latent_num_columns = latent_dims
        self.hidden_dims = hidden_dims
        self.action_dims = action_dims
        self.observation_dim_x, self.observation_dim_y = observation_dims
        self.horizon = training_horizon
        self.buckets = reward_buckets
        self.beta_pred, self.beta_dyn, self.beta_rep = beta_pred, beta_dyn, beta_rep
        self.batch_size = batch_size
        R, C = latent_dims
        self.encoder = Encoder(observation_dims, hidden_dims, R, C, num_encoder_filters_1, num_encoder_filters_2,
                               encoder_hidden_layer_nodes, device=device)
        self.sequence_model = SequenceModel(R, C, hidden_dims, action_dims, num_layers=1, device=device)
        self.dynamics_predictor = DynamicsPredictor(R, C, hidden_dims, dyn_pred_hidden_num_nodes_1,
                                                    dyn_pred_hidden_num_nodes_2, device)
        self.reward_predictor = RewardPredictor(R, C, hidden_dims, rew_pred_hidden_num_nodes_1,
                                                rew_pred_hidden_num_nodes_2, reward_buckets, device=device)
        self.continue_predictor = ContinuePredictor(R, C, hidden_dims, cont_pred_hidden_num_nodes_1,
                                                    cont_pred_hidden_num_nodes_2, device=device)
        self.decoder = Decoder(R, C, observation_dims, hidden_dims, num_decoder_filters_1, num_decoder_filters_2,
                               decoder_hidden_layer_nodes, device=device)
        self.device = torch.device(device)
        self.optimiser = torch.optim.AdamW(self.parameters(), lr=WM_lr, betas=(WM_betas[0], WM_betas[1]), eps=WM_eps,
                                           weight_decay=1e-6)
        self.scalar = torch.amp.GradScaler(enabled=self.device.type == "cuda")

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
        if agent is not None:
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
        L.call("dr_imagine_step", d, self.packed(), B, L.ptr(h), L.ptr(z), L.ptr(a), hip.rng(dev).noise(), L.ptr(h2),
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
               hip.rng(dev).noise(), L.ptr(z), L.ptr(h), L.ptr(lg), L.ptr(ws2), ws2.numel(), st)
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
        obs_ll = -(dec_mu.float() - obs_t.float()).pow(2).sum(dim=[-3, -2, -1])
        cont_ll = torch.nn.functional.binary_cross_entropy_with_logits(cont_logits, cont_t, reduction="none")
        rew_ll = torch.sum(to_twohot(rew_t, self.reward_predictor.buckets_rew)
                           * torch.nn.functional.log_softmax(reward_logits, dim=-1), dim=-1, keepdim=True)
        return prior_logits[:, 1:], post_logits[:, 1:], obs_ll[:, 1:], rew_ll, cont_ll

    def training_step(self, observation_sequences, action_sequences, reward_sequences, continue_sequences):
        """WorldModel.training_step (WorldModel.py:148-202)."""
        obs = (observation_sequences.float() / 255.0) - 0.5
        H = self.horizon
        dev_type = self.device.type
        with torch.autocast(device_type=dev_type, dtype=torch.float16):
            prior_l, post_l, obs_ll, rew_ll, cont_ll = self.unroll_model(
                obs[:, :H], action_sequences[:, :H], reward_sequences[:, :H], continue_sequences[:, :H])
            mask = continue_sequences[:, :H - 1]
            obs_ll = obs_ll * mask.squeeze(-1)
            rew_ll = rew_ll * mask
            cont_ll = cont_ll * mask
            Cat = torch.distributions.Categorical
            kl = torch.distributions.kl.kl_divergence
            kl_dyn = kl(Cat(logits=post_l.detach().float()), Cat(logits=prior_l.float())).sum(dim=-1)
            kl_rep = kl(Cat(logits=post_l.float()), Cat(logits=prior_l.detach().float())).sum(dim=-1)
            kl_dyn = torch.mean(kl_dyn * mask.squeeze(-1))
            kl_rep = torch.mean(kl_rep * mask.squeeze(-1))
            denom = mask.sum() + 1e-5
            loss_pred = (-obs_ll.sum() - rew_ll.sum() + cont_ll.sum()) / denom
            one = torch.tensor(1.0, device=obs.device)
            total = self.beta_pred * loss_pred + self.beta_dyn * torch.max(one, kl_dyn) + \
                self.beta_rep * torch.max(one, kl_rep)
            if torch.isnan(total) or torch.isinf(total):
                print("World Model loss is nan or inf, skipping update.")
                return total
        self.optimiser.zero_grad()
        self.scalar.scale(total).backward()
        self.scalar.unscale_(self.optimiser)
        nn.utils.clip_grad_norm_(self.parameters(), 100.0)
        self.scalar.step(self.optimiser)
        self.scalar.update()
        return total
