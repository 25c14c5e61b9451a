"""World-model networks with the reference's module/parameter names
(state_dict-compatible with SequenceModel.py, DynamicsPredictors.py and
VariationalAutoEncoder.py), so reference checkpoints load unchanged.

Two execution paths, chosen per call:
  * inference calls (no autograd through the weights) run the hand-written
    HIP kernels of libdreamer_hip -- the imagination hot path;
  * calls that need autograd through the world-model weights (only
    WorldModel.training_step, SURVEY §8f "next") use the nn.Modules' own
    forward on the GPU.
Hot-path methods raise on CPU tensors: there is no CPU fallback."""
import torch
import torch.nn as nn

from . import _lib as L
from . import hip


def _mlp3(n_in, h1, h2, n_out, device):
    """Linear-LN-SiLU-Linear-LN-SiLU-Linear (Sequential indices 0,1,3,4,6)."""
    return nn.Sequential(
        nn.Linear(n_in, h1, device=device), nn.LayerNorm(h1, device=device), nn.SiLU(),
        nn.Linear(h1, h2, device=device), nn.LayerNorm(h2, device=device), nn.SiLU(),
        nn.Linear(h2, n_out, device=device))


def _mlp_dims(seq):
    return seq[0].in_features, seq[0].out_features, seq[3].out_features, seq[6].out_features


def run_mlp3(seq, h, z=None):
    """HIP forward of a _mlp3 on [h | flatten(z)] -> (M, n_out)."""
    L.require_gpu(h)
    n_in, h1, h2, n_out = _mlp_dims(seq)
    lead = h.shape[:-1]
    hh = h.reshape(-1, h.shape[-1]).contiguous()
    M = hh.shape[0]
    zz = None if z is None else z.reshape(M, -1).contiguous()
    out = torch.empty(M, n_out, device=h.device)
    ws = hip.workspace(h.device).get("mlp3", 4 * M * (h1 + h2) + 1024)
    L.call("dr_mlp3_fwd", hip.mlp3(seq), M, hh.shape[1], L.ptr(hh), hh.shape[1],
           0 if zz is None else zz.shape[1], L.ptr(zz), 0 if zz is None else zz.shape[1], h1, h2, n_out,
           L.ptr(out), n_out, L.ptr(ws), ws.numel(), hip.stream())
    return out.view(*lead, n_out)


class SequenceModel(nn.Module):
    """RSSM deterministic core: GRUCell(R*C + A -> hidden) on cat(flatten(z), a)
    (SequenceModel.py:4-24)."""

    def __init__(self, latent_num_rows, latent_num_columns, hidden_dim, action_dim, *, num_layers=1, device="cpu"):
        super().__init__()
        self.latent_dim = latent_num_rows * latent_num_columns
        self.hidden_dim = hidden_dim
        self.action_dim = action_dim
        self.num_layers = num_layers
        self.device = device
        self.flatten = nn.Flatten(start_dim=2)
        self.GRU = nn.GRUCell(input_size=self.latent_dim + action_dim, hidden_size=hidden_dim, device=device)

    def dims(self):
        d = L.dr_dims()
        d.hidden, d.rows, d.cols, d.action = self.hidden_dim, self.latent_dim, 1, self.action_dim
        return d

    def packed(self):
        wm = L.dr_world_model()
        g = self.GRU
        wm.w_ih, wm.w_hh, wm.b_ih, wm.b_hh = (L.ptr(t) for t in (g.weight_ih, g.weight_hh, g.bias_ih, g.bias_hh))
        return wm

    def forward(self, last_latent_state, last_hidden_state, last_action):
        if hip.needs_torch_grad(self):
            x = torch.cat((self.flatten(last_latent_state), last_action), dim=-1).squeeze(1)
            return self.GRU(x, last_hidden_state.squeeze(1)).unsqueeze(1)
        L.require_gpu(last_hidden_state)
        B = last_hidden_state.shape[0]
        z = last_latent_state.reshape(B, -1).contiguous()
        h = last_hidden_state.reshape(B, -1).contiguous()
        a = last_action.reshape(B, -1).contiguous()
        out = torch.empty(B, 1, self.hidden_dim, device=h.device)
        ws = hip.workspace(h.device).get("gru", 4 * 6 * B * self.hidden_dim + 1024)
        d = self.dims()
        L.call("dr_gru_cell", d, self.packed(), B, L.ptr(z), L.ptr(h), L.ptr(a), L.ptr(out), L.ptr(ws), ws.numel(),
               hip.stream())
        return out


class DynamicsPredictor(nn.Module):
    """Prior p(z|h): MLP -> (R,C) logits; unimix categorical sample with STE
    (DynamicsPredictors.py:5-40)."""

    def __init__(self, latent_num_rows, latent_num_columns, hidden_state_size, hidden_L1, hidden_L2, device):
        super().__init__()
        self.latent_num_rows, self.latent_num_columns = latent_num_rows, latent_num_columns
        self.latent_size = latent_num_rows * latent_num_columns
        self.device = device
        self.logit_net = _mlp3(hidden_state_size, hidden_L1, hidden_L2, self.latent_size, device)

    def forward(self, x):
        if hip.needs_torch_grad(self):
            lg = self.logit_net(x)
        else:
            lg = run_mlp3(self.logit_net, x)
        return lg.view(*x.shape[:-1], self.latent_num_rows, self.latent_num_columns)

    def predict(self, hidden_state):
        if hip.needs_torch_grad(self):
            raise RuntimeError("DynamicsPredictor.predict with autograd through the prior is not part of the "
                               "imagination path; use WorldModel.training_step or no_grad")
        logits = self.forward(hidden_state)
        return sample_latent(logits, self.latent_num_rows, self.latent_num_columns), logits


def sample_latent(logits, rows, cols, noise=None):
    """HIP categorical sample (one-hot + STE value) of logits (..., R, C)."""
    L.require_gpu(logits)
    lead = logits.shape[:-2]
    lg = logits.reshape(-1, rows * cols).contiguous().float()
    M = lg.shape[0]
    z = torch.empty(M, rows * cols, device=lg.device)
    nz = noise if noise is not None else hip.adhoc(lg.device).noise()
    L.call("dr_categorical_sample", M, rows, cols, L.ptr(lg), nz, L.ptr(z), None, None, hip.stream())
    return z.view(*lead, rows, cols)


class RewardPredictor(nn.Module):
    """Reward head: MLP on cat(h, z) -> 255 two-hot buckets; value =
    symexp(E[bucket]) (DynamicsPredictors.py:42-74)."""

    def __init__(self, latent_num_rows, latent_num_columns, hidden_state_size, hidden_L1, hidden_L2, num_buckets=255,
                 device="cpu"):
        super().__init__()
        self.latent_size = latent_num_rows * latent_num_columns
        self.buckets = num_buckets
        self.device = device
        self.flatten = nn.Flatten(start_dim=2)
        self.logit_net = _mlp3(hidden_state_size + self.latent_size, hidden_L1, hidden_L2, num_buckets, device)
        self.register_buffer("buckets_rew", torch.linspace(-20.0, 20.0, num_buckets, device=device))

    def forward(self, hidden, latent):
        if hip.needs_torch_grad(self):
            return self.logit_net(torch.cat([hidden, self.flatten(latent)], dim=-1))
        return run_mlp3(self.logit_net, hidden, latent)

    def predict(self, hidden_state, latent_state):
        lg = self.forward(hidden_state, latent_state)
        if hip.needs_torch_grad(self):
            raise RuntimeError("RewardPredictor.predict under autograd is not on the imagination path")
        flat = lg.reshape(-1, self.buckets).contiguous()
        out = torch.empty(flat.shape[0], device=lg.device)
        L.call("dr_bucket_value", flat.shape[0], self.buckets, L.ptr(flat), L.ptr(self.buckets_rew), L.ptr(out),
               hip.stream())
        return out.view(*lg.shape[:-1], 1)


class ContinuePredictor(nn.Module):
    """Continue head: MLP on cat(h, z) -> 1 logit; sigmoid probability
    (DynamicsPredictors.py:76-105)."""

    def __init__(self, latent_num_rows, latent_num_columns, hidden_state_size, hidden_L1, hidden_L2, device):
        super().__init__()
        self.latent_size = latent_num_rows * latent_num_columns
        self.device = device
        self.flatten = nn.Flatten(start_dim=2)
        self.logit_generator = _mlp3(hidden_state_size + self.latent_size, hidden_L1, hidden_L2, 1, device)

    def forward(self, hidden, latent):
        if hip.needs_torch_grad(self):
            logit = self.logit_generator(torch.cat([hidden, self.flatten(latent)], dim=-1))
        else:
            logit = run_mlp3(self.logit_generator, hidden, latent)
        return torch.sigmoid(logit), logit

    def predict(self, hidden_state, latent_state):
        prob, _ = self.forward(hidden_state, latent_state)
        return prob


def vae_channels(depth, f1, f2):
    """Encoder channels 3, f1, f2, 2 f2, 4 f2 (VariationalAutoEncoder.py:33-42); depth 5 (BASELINE
    configs[3]'s "deeper VAE", config key encoder_depth) adds one 4 f2 -> 4 f2 stride-2 layer
    (include/dreamer_hip.h dr_dims.enc_depth)."""
    if depth not in (4, 5):
        raise ValueError(f"encoder_depth must be 4 (the reference) or 5 (the deeper VAE), got {depth}")
    return [3, f1, f2, 2 * f2, 4 * f2] + ([4 * f2] if depth == 5 else [])


class Encoder(nn.Module):
    """4x [Conv2d(k4,s2,p1)+SiLU] -> flatten -> cat(features, h) -> Linear-LN-SiLU
    -> Linear -> (R,C) logits; unimix categorical sample + STE
    (VariationalAutoEncoder.py:4-99).  depth=5: one more stride-2 conv (configs[3])."""

    def __init__(self, observation_dims, hidden_state_dim, latent_num_rows, latent_num_columns, num_filters_1,
                 num_filters_2, hidden_layer_nodes, device="cpu", depth=4):
        super().__init__()
        self.depth = int(depth)
        self.latent_size = latent_num_rows * latent_num_columns
        self.latent_num_rows, self.latent_num_columns = latent_num_rows, latent_num_columns
        self.observation_dims = tuple(observation_dims)
        self.hidden_state_dim = hidden_state_dim
        self.num_filters_1 = num_filters_1
        # observation_dims = [D]: proprioceptive vector observations (BASELINE
        # configs[4]).  The reference encoder is always convolutional
        # (VAE.py:33-42); the stand-in is Linear(D, 4 f2)-SiLU-Linear(4 f2, 4 f2)-SiLU
        # with the same latent_mapper (include/dreamer_hip.h dr_dims.obs_dim).
        self.vector = len(self.observation_dims) == 1
        if self.vector:
            D, F = self.observation_dims[0], 4 * num_filters_2
            self.final_height = self.final_width = 1
            self.feature_extractor = nn.Sequential(nn.Linear(D, F, device=device), nn.SiLU(),
                                                   nn.Linear(F, F, device=device), nn.SiLU())
            n_feat = F
        else:
            chans = vae_channels(self.depth, num_filters_1, num_filters_2)
            self.final_height = observation_dims[0] // 2 ** self.depth
            self.final_width = observation_dims[1] // 2 ** self.depth
            if self.final_height < 1 or self.final_width < 1:
                raise ValueError(f"Input image {observation_dims} is too small for {self.depth} layers of downsampling.")
            layers = []
            for cin, cout in zip(chans[:-1], chans[1:]):
                layers += [nn.Conv2d(cin, cout, kernel_size=4, stride=2, padding=1, device=device), nn.SiLU()]
            self.feature_extractor = nn.Sequential(*layers)
            n_feat = chans[-1] * self.final_height * self.final_width
        self.flatten = nn.Flatten(start_dim=2)
        self.latent_mapper = nn.Sequential(
            nn.Linear(n_feat + hidden_state_dim, hidden_layer_nodes, device=device),
            nn.LayerNorm(hidden_layer_nodes, device=device), nn.SiLU(),
            nn.Linear(hidden_layer_nodes, self.latent_size, device=device))

    # -- packing for libdreamer_hip -------------------------------------------
    def fill_dims(self, d):
        if self.vector:
            d.img_h = d.img_w = 0
            d.obs_dim = self.observation_dims[0]
            d.enc_f1 = self.num_filters_1
            d.enc_f2 = self.feature_extractor[0].out_features // 4
        else:
            d.img_h, d.img_w = self.observation_dims
            d.obs_dim = 0
            d.enc_f1 = self.feature_extractor[0].out_channels
            d.enc_f2 = self.feature_extractor[2].out_channels
            d.enc_depth = self.depth
        d.enc_hidden = self.latent_mapper[0].out_features
        d.hidden = self.hidden_state_dim
        d.rows, d.cols = self.latent_num_rows, self.latent_num_columns

    def fill(self, wm):
        fe = self.feature_extractor
        for i in range(len(fe) // 2):
            wm.conv[i] = hip.linear(fe[2 * i])
        wm.map0, wm.map1, wm.map3 = (hip.linear(self.latent_mapper[j]) for j in (0, 1, 3))

    def forward(self, hidden, observation):
        B, S = observation.shape[:2]
        if hip.needs_torch_grad(self) and self.vector:
            feat = self.feature_extractor(observation.reshape(B, S, -1))
            return self.latent_mapper(torch.cat((feat, hidden), dim=-1))
        if hip.needs_torch_grad(self):
            C, H, W = observation.shape[2:]
            feat = self.feature_extractor(observation.reshape(B * S, C, H, W))
            feat = self.flatten(feat.view(B, S, *feat.shape[1:]))
            return self.latent_mapper(torch.cat((feat, hidden), dim=-1))
        logits, _ = self._hip(hidden, observation, sample=False)
        return logits.view(B, S, -1)

    def _hip(self, hidden, observation, sample, noise=None, raw255=False):
        L.require_gpu(observation)
        B, S = observation.shape[:2]
        n = B * S
        dev = observation.device
        d = L.dr_dims()
        self.fill_dims(d)
        wm = L.dr_world_model()
        self.fill(wm)
        obs = observation.reshape(n, -1).float().contiguous()
        fr = L.dr_frames(None, 0, None, L.ptr(obs), obs.shape[1], 0, 1 if raw255 else 0)
        eh = d.enc_hidden
        feat = torch.empty(n, eh, device=dev)
        wsz = L.query("dr_encoder_workspace_bytes", d, n)
        ws = hip.workspace(dev).get("enc", wsz)
        st = hip.stream()
        L.call("dr_encoder_features", d, wm, fr, n, 1, L.ptr(feat), L.ptr(ws), ws.numel(), st)
        h = hidden.reshape(n, -1).float().contiguous()
        z = torch.empty(n, self.latent_size, device=dev)
        logits = torch.empty(n, self.latent_size, device=dev)
        ws2 = hip.workspace(dev).get("obs", L.query("dr_observe_workspace_bytes", d, n))
        nz = noise if noise is not None else hip.adhoc(dev).noise()
        hout = torch.empty_like(h)
        L.call("dr_observe_scan", d, wm, n, 1, L.ptr(feat), None, 0, 0, L.ptr(h), None, nz, L.ptr(z), L.ptr(hout),
               L.ptr(logits), L.ptr(ws2), ws2.numel(), st)
        return logits, z

    def encode(self, hidden_state, observation):
        B, S, _ = hidden_state.shape
        if hip.needs_torch_grad(self):
            raise RuntimeError("Encoder.encode under autograd is only used by WorldModel.training_step")
        logits, z = self._hip(hidden_state, observation, sample=True)
        R, C = self.latent_num_rows, self.latent_num_columns
        return z.view(B, S, R, C), logits.view(B, S, R, C)


class Decoder(nn.Module):
    """cat(h, z) -> Linear-LN-SiLU -> Linear-SiLU -> 4x ConvTranspose2d (SiLU,
    Tanh out) (VariationalAutoEncoder.py:101-166).  Inference runs
    dr_decoder_fwd (parity-class transposed-conv implicit GEMMs, direct
    3-channel output kernel); the world-model training step runs the decoder
    inside dr_wm_train_grads.  Autograd callers get the nn.Module forward."""

    def __init__(self, latent_num_rows, latent_num_columns, observation_dim, hidden_state_dim, num_filters_1,
                 num_filters_2, hidden_layer_nodes, device="cpu", depth=4):
        super().__init__()
        # observation_dim = [D]: vector observations (Encoder's note); the
        # image_builder stand-in is Linear(4 f2, 4 f2)-SiLU-Linear(4 f2, D), no Tanh
        self.vector = len(observation_dim) == 1
        self.observation_dim = tuple(observation_dim)
        self.num_filters_1, self.num_filters_2 = num_filters_1, num_filters_2
        self.depth = int(depth)
        self.start_height = 1 if self.vector else observation_dim[0] // 2 ** self.depth
        self.start_width = 1 if self.vector else observation_dim[1] // 2 ** self.depth
        self.num_filters_start = num_filters_2 * 4
        self.hidden_dim = hidden_state_dim
        self.latent_row_dim, self.latent_col_dim = latent_num_rows, latent_num_columns
        self.flatten = nn.Flatten(start_dim=1)
        n_start = self.num_filters_start * self.start_height * self.start_width
        self.upscaler = nn.Sequential(
            nn.Linear(latent_num_rows * latent_num_columns + hidden_state_dim, hidden_layer_nodes, device=device),
            nn.LayerNorm(hidden_layer_nodes, device=device), nn.SiLU(),
            nn.Linear(hidden_layer_nodes, n_start, device=device), nn.SiLU())
        if self.vector:
            self.image_builder = nn.Sequential(nn.Linear(n_start, n_start, device=device), nn.SiLU(),
                                               nn.Linear(n_start, observation_dim[0], device=device))
            return
        # the encoder's channels mirrored (VAE.py:128-137; depth 5: the deeper VAE's extra 4 f2 -> 4 f2 layer)
        chans = [c for c in reversed(vae_channels(self.depth, num_filters_1, num_filters_2))]
        chans[0] = self.num_filters_start
        layers = []
        for i, (cin, cout) in enumerate(zip(chans[:-1], chans[1:])):
            layers.append(nn.ConvTranspose2d(cin, cout, kernel_size=4, stride=2, padding=1, device=device))
            layers.append(nn.Tanh() if i == self.depth - 1 else nn.SiLU())
        self.image_builder = nn.Sequential(*layers)

    def fill_dims(self, d):
        d.dec_f1, d.dec_f2 = self.num_filters_1, self.num_filters_2
        d.dec_hidden = self.upscaler[0].out_features
        if self.vector:
            d.obs_dim = self.observation_dim[0]
            d.img_h = d.img_w = 0
        else:
            d.obs_dim = 0
            d.enc_depth = self.depth
            d.img_h, d.img_w = 2 ** self.depth * self.start_height, 2 ** self.depth * self.start_width

    def packed(self):
        ib = self.image_builder
        dec = L.dr_decoder(hip.linear(self.upscaler[0]), hip.linear(self.upscaler[1]), hip.linear(self.upscaler[3]))
        for i in range((len(ib) + 1) // 2):
            dec.convt[i] = hip.linear(ib[2 * i])
        return dec

    def forward(self, hidden, latent):
        B, S, _ = hidden.shape
        if not hip.needs_torch_grad(self):
            return self._hip(hidden, latent)
        x = torch.cat((hidden.reshape(B * S, self.hidden_dim), self.flatten(latent.reshape(B * S, -1))), dim=-1)
        if self.vector:
            return self.image_builder(self.upscaler(x)).view(B, S, -1)
        x = self.upscaler(x).view(-1, self.num_filters_start, self.start_height, self.start_width)
        mu = self.image_builder(x)
        return mu.view(B, S, *mu.shape[1:])

    def _hip(self, hidden, latent):
        L.require_gpu(hidden)
        B, S, _ = hidden.shape
        M = B * S
        h = hidden.reshape(M, self.hidden_dim).float().contiguous()
        z = latent.reshape(M, -1).float().contiguous()
        d = L.dr_dims()
        d.hidden, d.rows, d.cols = self.hidden_dim, self.latent_row_dim, self.latent_col_dim
        self.fill_dims(d)
        dec = self.packed()
        mu = torch.empty(B, S, *((d.obs_dim,) if self.vector else (3, d.img_h, d.img_w)), device=h.device)
        ws = hip.workspace(h.device).get("dec", L.query("dr_decoder_workspace_bytes", d, M))
        L.call("dr_decoder_fwd", d, dec, M, L.ptr(h), h.shape[1], L.ptr(z), z.shape[1], L.ptr(mu), L.ptr(ws),
               ws.numel(), hip.stream())
        return mu

    def decode(self, hidden_state, latent_state):
        return self.forward(hidden_state, latent_state)
