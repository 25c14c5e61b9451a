"""Actor-critic with the reference's API and parameter names (Agent.py).

Parameters of the actor, the critic and the target critic live in flat
device buffers (the nn.Parameters are views into them, so state_dict and
load_state_dict behave as in the reference); their gradients live in ONE flat
buffer [actor | critic | 2 loss slots] so a data-parallel step is a single
all-reduce.  AdamW, clip_grad_norm_ and the soft target update are fused
flat-buffer HIP kernels."""
import copy

import torch
import torch.nn as nn

from . import _lib as L
from . import hip


class _Flat:
    """Rebinds a module's parameters as views into one flat buffer."""

    def __init__(self, module, grad_storage=None):
        self.module = module
        self.rebind(grad_storage)

    def rebind(self, grad_storage=None):
        named = list(self.module.named_parameters())
        self.names = [n for n, _ in named]
        self.params = [p for _, p in named]
        # every parameter starts on a 256-byte boundary (float4 weight rows for
        # the skinny GEMM); the pad elements stay 0 (zero grad -> AdamW no-op)
        self.offsets, off = {}, 0
        for name, p in named:
            self.offsets[name] = off
            off += -(-p.numel() // 64) * 64
        n = off
        dev = self.params[0].device
        self.flat = torch.zeros(n, device=dev, dtype=torch.float32)
        for name, p in named:
            o, k = self.offsets[name], p.numel()
            self.flat[o:o + k].copy_(p.data.reshape(-1))
            p.data = self.flat[o:o + k].view_as(p)
        self.numel = n
        self.grad = grad_storage if grad_storage is not None else torch.zeros(n, device=dev)
        self.bind_grads()

    def bind_grads(self):
        for name, p in zip(self.names, self.params):
            o = self.offsets[name]
            p.grad = self.grad[o:o + p.numel()].view_as(p)

    def intact(self):
        base = self.flat.data_ptr()
        return all(p.data_ptr() == base + 4 * self.offsets[n] for n, p in zip(self.names, self.params))

    def sync_grads(self):
        """After a PyTorch autograd pass: move grads that autograd stored in
        fresh tensors back into the flat buffer."""
        for name, p in zip(self.names, self.params):
            o = self.offsets[name]
            view = self.grad[o:o + p.numel()].view_as(p)
            if p.grad is None:
                view.zero_()
            elif p.grad.data_ptr() != view.data_ptr():
                view.copy_(p.grad)
            p.grad = view

    def ptr(self, name, grad=False):
        t = self.grad if grad else self.flat
        return t.data_ptr() + 4 * self.offsets[name]


class FlatAdamW(torch.optim.AdamW):
    """torch.optim.AdamW over a _Flat buffer, stepped by the fused HIP kernel
    (same op order as torch's single-tensor AdamW; step counter on device)."""

    def __init__(self, flat, lr, betas, eps, weight_decay):
        super().__init__(flat.params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        self.flat_ref = flat
        dev = flat.flat.device
        self.exp_avg = torch.zeros(flat.numel, device=dev)
        self.exp_avg_sq = torch.zeros(flat.numel, device=dev)
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self.hyper = torch.zeros(2, device=dev)

    def fused_step(self, sqnorm=None, max_norm=100.0, skip=None):
        g = self.param_groups[0]
        f = self.flat_ref
        L.call("dr_adamw", f.numel, f.flat.data_ptr(), f.grad.data_ptr(), self.exp_avg.data_ptr(),
               self.exp_avg_sq.data_ptr(), None if sqnorm is None else sqnorm.data_ptr(), max_norm, g["lr"],
               g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"], self.step_dev.data_ptr(),
               self.hyper.data_ptr(), None if skip is None else skip.data_ptr(), hip.stream())

    @torch.no_grad()
    def step(self, closure=None):
        if not self.flat_ref.flat.is_cuda:
            raise RuntimeError("dreamer_amd optimisers run on the GPU only")
        self.flat_ref.sync_grads()
        self.fused_step()

    def zero_grad(self, set_to_none=True):
        self.flat_ref.grad.zero_()
        self.flat_ref.bind_grads()


class Actor(nn.Module):
    """tanh-Normal policy on cat(h, flatten(z)) (Agent.py:174-210)."""

    def __init__(self, action_dim, latent_column_dim, latent_row_dim, hidden_state_dim, hidden_layer_num_nodes_1,
                 hidden_layer_num_nodes_2, *, device="cpu"):
        super().__init__()
        self.action_dim = action_dim
        self.flatten = nn.Flatten(start_dim=2)
        n_in = latent_row_dim * latent_column_dim + hidden_state_dim
        h1, h2 = hidden_layer_num_nodes_1, hidden_layer_num_nodes_2
        self.base_net = nn.Sequential(nn.Linear(n_in, h1, device=device), nn.LayerNorm(h1, device=device), nn.SiLU(),
                                      nn.Linear(h1, h2, device=device), nn.LayerNorm(h2, device=device), nn.SiLU())
        self.mu_head = nn.Linear(h2, action_dim, device=device)
        self.log_sig_head = nn.Linear(h2, action_dim, device=device)
        nn.init.zeros_(self.mu_head.weight)
        nn.init.zeros_(self.mu_head.bias)
        self._agent = None

    def forward(self, ht, zt):
        x = self.base_net(torch.cat([ht, self.flatten(zt)], dim=-1))
        ls = torch.clamp(self.log_sig_head(x), -5.0, 2.0)
        return self.mu_head(x), torch.nn.functional.softplus(ls) + 1e-3

    def act(self, ht, zt, deterministic=False):
        if hip.needs_torch_grad(self):
            mu, sigma = self.forward(ht, zt)
            if deterministic:
                return torch.tanh(mu), mu, sigma
            return torch.tanh(mu + torch.randn_like(mu) * sigma), mu, sigma
        L.require_gpu(ht)
        lead = ht.shape[:-1]
        B = ht[..., 0].numel()
        h = ht.reshape(B, -1).contiguous()
        z = zt.reshape(B, -1).contiguous()
        A = self.action_dim
        a, mu, sg = (torch.empty(B, A, device=h.device) for _ in range(3))
        d = self._dims(h.shape[1], z.shape[1])
        ws = hip.workspace(h.device).get("act", L.query("dr_actor_act_workspace_bytes", d, B))
        L.call("dr_actor_act", d, self.struct(), B, L.ptr(h), L.ptr(z), hip.adhoc(h.device).noise(),
               int(deterministic), L.ptr(a), L.ptr(mu), L.ptr(sg), L.ptr(ws), ws.numel(), hip.stream())
        return a.view(*lead, A), mu.view(*lead, A), sg.view(*lead, A)

    def _dims(self, hidden, latent):
        d = L.dr_dims()
        d.hidden, d.rows, d.cols, d.action = hidden, latent, 1, self.action_dim
        d.actor_h1, d.actor_h2 = self.base_net[0].out_features, self.base_net[3].out_features
        return d

    def struct(self):
        b = self.base_net
        return L.dr_actor(hip.linear(b[0]), hip.linear(b[1]), hip.linear(b[3]), hip.linear(b[4]),
                          hip.linear(self.mu_head), hip.linear(self.log_sig_head))


class Critic(nn.Module):
    """255-bucket two-hot value head on cat(h, flatten(z)) (Agent.py:212-241)."""

    def __init__(self, latent_row_dim, latent_column_dim, hidden_state_dim, hidden_layer_num_nodes_1,
                 hidden_layer_num_nodes_2, num_buckets=255, device="cpu"):
        super().__init__()
        self.latent_row_dim, self.latent_column_dim = latent_row_dim, latent_column_dim
        self.num_buckets = num_buckets
        self.flatten = nn.Flatten(start_dim=2)
        n_in = latent_column_dim * latent_row_dim + hidden_state_dim
        h1, h2 = hidden_layer_num_nodes_1, hidden_layer_num_nodes_2
        self.value_net = nn.Sequential(nn.Linear(n_in, h1, device=device), nn.LayerNorm(h1, device=device), nn.SiLU(),
                                       nn.Linear(h1, h2, device=device), nn.LayerNorm(h2, device=device), nn.SiLU(),
                                       nn.Linear(h2, num_buckets, device=device))
        self.register_buffer("buckets_crit", torch.linspace(-20, 20, num_buckets, device=device))

    def forward(self, ht, zt):
        if hip.needs_torch_grad(self):
            return self.value_net(torch.cat([ht, self.flatten(zt)], dim=-1))
        return self._hip(ht, zt, want_logits=True)[0]

    def value(self, ht, zt):
        if hip.needs_torch_grad(self):
            probs = torch.softmax(self.forward(ht, zt), dim=-1)
            v = torch.sum(probs * self.buckets_crit, dim=-1, keepdim=True)
            return torch.sign(v.clamp(-20, 20)) * (torch.exp(v.clamp(-20, 20).abs()) - 1.0)
        return self._hip(ht, zt, want_logits=False)[1]

    def _hip(self, ht, zt, want_logits):
        L.require_gpu(ht)
        lead = ht.shape[:-1]
        M = ht[..., 0].numel()
        h = ht.reshape(M, -1).contiguous()
        z = zt.reshape(M, -1).contiguous()
        d = L.dr_dims()
        d.hidden, d.rows, d.cols = h.shape[1], z.shape[1], 1
        d.critic_h1, d.critic_h2 = self.value_net[0].out_features, self.value_net[3].out_features
        d.buckets = self.num_buckets
        lg = torch.empty(M, self.num_buckets, device=h.device) if want_logits else None
        v = torch.empty(M, device=h.device)
        ws = hip.workspace(h.device).get("crit", L.query("dr_critic_tape_bytes", d, M))
        L.call("dr_critic_fwd", d, self.struct(), M, L.ptr(h), h.shape[1], L.ptr(z), z.shape[1], L.ptr(lg), L.ptr(v),
               None, L.ptr(ws), ws.numel(), hip.stream())
        return (None if lg is None else lg.view(*lead, -1)), v.view(*lead, 1)

    def struct(self):
        return L.dr_critic(hip.mlp3(self.value_net), L.ptr(self.buckets_crit))


class Agent(nn.Module):
    """Actor, critic, EMA target critic, return normaliser S and their
    optimisers (Agent.py:7-172)."""

    def __init__(self, action_dim, latent_dims, hidden_state_dim, HL_A1, HL_A2, HL_C1, HL_C2, critic_buckets, A_lr,
                 A_betas, A_eps, C_lr, C_betas, C_eps, nu, lambda_, gamma, *, device="cpu"):
        super().__init__()
        self.device = torch.device(device)
        self.actor = Actor(action_dim, latent_dims[0], latent_dims[1], hidden_state_dim, HL_A1, HL_A2, device=device)
        self.critic = Critic(latent_dims[0], latent_dims[1], hidden_state_dim, HL_C1, HL_C2, critic_buckets,
                             device=device)
        self.target_critic = copy.deepcopy(self.critic)
        for p in self.target_critic.parameters():
            p.requires_grad = False
        self.nu, self.lambda_, self.gamma = nu, lambda_, gamma
        self.buckets = critic_buckets
        self.smoothing_factor = 0.99
        self.S_dev = torch.ones((), device=self.device)
        # False after a persistent-kernel fault: every entry point then runs its launch form
        self.persistent_ok = True
        self._A_hp = (A_lr, tuple(A_betas), A_eps)
        self._C_hp = (C_lr, tuple(C_betas), C_eps)
        self._flat = None
        self._bind()

    # ---- flat buffers --------------------------------------------------------
    def _bind(self):
        pad = lambda m: sum(-(-p.numel() // 64) * 64 for p in m.parameters())
        na, nc = pad(self.actor), pad(self.critic)
        # [actor grads | critic grads | actor loss, critic loss, fault]: the fault
        # slot (dr_dims.fault) turns NaN when a persistent kernel timed out; it
        # rides in the flat buffer's all-reduce (every rank sees it) and in the
        # optimiser's non-finite check (the update is skipped, Agent.py:137-139)
        self.grad_buffer = torch.zeros(na + nc + 3, device=self.device)
        self.loss_buffer = self.grad_buffer[na + nc:]
        self.fa = _Flat(self.actor, self.grad_buffer[:na])
        self.fc = _Flat(self.critic, self.grad_buffer[na:na + nc])
        self.ft = _Flat(self.target_critic, torch.zeros(nc, device=self.device))
        (alr, ab, ae), (clr, cb, ce) = self._A_hp, self._C_hp
        self.actor_optimiser = FlatAdamW(self.fa, alr, ab, ae, 1e-6)
        self.critic_optimiser = FlatAdamW(self.fc, clr, cb, ce, 1e-6)
        self._flat = True

    def _ensure_flat(self):
        if not (self.fa.intact() and self.fc.intact() and self.ft.intact()):
            self.fa.rebind(self.fa.grad)
            self.fc.rebind(self.fc.grad)
            self.ft.rebind(self.ft.grad)

    def params_key(self):
        self._ensure_flat()
        return (self.fa.flat.data_ptr(), self.fc.flat.data_ptr(), self.ft.flat.data_ptr(),
                self.grad_buffer.data_ptr())

    def loss_slot(self, i):
        return self.loss_buffer[i:i + 1]

    def fault_slot(self):
        """Device float, NaN once a persistent kernel timed out (sticky until the
        host acknowledges it, engine.ImaginationEngine.check_faults)."""
        return self.loss_buffer[2:3]

    def fault_host(self):
        """(pinned host int32 [1], its device address): set to 1 by the kernel
        that timed out, read by the host without a copy or a sync."""
        if getattr(self, "_fault_host", None) is None:
            import ctypes
            h = torch.zeros(1, dtype=torch.int32).pin_memory()
            p = ctypes.c_void_p()
            L.call("dr_host_device_ptr", h.data_ptr(), ctypes.byref(p))
            self._fault_host = (h, p.value)
        return self._fault_host

    @property
    def S(self):
        return self.S_dev

    @S.setter
    def S(self, v):
        self.S_dev.fill_(float(v))

    def actor_struct(self, grad=False):
        f = self.fa
        g = lambda n: f.ptr(n, grad)
        return L.dr_actor(L.dr_linear(g("base_net.0.weight"), g("base_net.0.bias")),
                          L.dr_linear(g("base_net.1.weight"), g("base_net.1.bias")),
                          L.dr_linear(g("base_net.3.weight"), g("base_net.3.bias")),
                          L.dr_linear(g("base_net.4.weight"), g("base_net.4.bias")),
                          L.dr_linear(g("mu_head.weight"), g("mu_head.bias")),
                          L.dr_linear(g("log_sig_head.weight"), g("log_sig_head.bias")))

    def critic_struct(self, target=False, grad=False):
        f = self.ft if target else self.fc
        g = lambda n: f.ptr(n, grad)
        lin = lambda i: L.dr_linear(g(f"value_net.{i}.weight"), g(f"value_net.{i}.bias"))
        net = L.dr_mlp3(lin(0), lin(1), lin(3), lin(4), lin(6))
        mod = self.target_critic if target else self.critic
        return L.dr_critic(net, L.ptr(mod.buckets_crit))

    # ---- optimiser -----------------------------------------------------------
    def fused_optimiser_step(self, sq, skip):
        """NaN/Inf loss -> skip (Agent.py:137-139), clip_grad_norm_(100) per
        network (Agent.py:147-148), AdamW steps (150-151), target EMA (153)."""
        st = hip.stream()
        if getattr(self, "_clip_scratch", None) is None or self._clip_scratch.device != sq.device:
            self._clip_scratch = torch.zeros(1024, device=sq.device)  # DR_CLIP_SCRATCH_FLOATS
        # critic / actor AdamW (clip by sq[1] / sq[0]) and the target EMA
        # (tau = 0.02, Agent.py:90-94) in one more launch: dr_ac_optimiser_step
        # = dr_clip_stats + dr_adamw x2 + dr_ema, the same bits
        ca, oa, tau = self.critic_optimiser, self.actor_optimiser, 0.02
        ga, gc = oa.param_groups[0], ca.param_groups[0]
        L.call("dr_ac_optimiser_step",
               self.fa.numel, self.fa.flat.data_ptr(), self.fa.grad.data_ptr(), oa.exp_avg.data_ptr(),
               oa.exp_avg_sq.data_ptr(), oa.step_dev.data_ptr(), oa.hyper.data_ptr(), ga["lr"], ga["betas"][0],
               ga["betas"][1], ga["eps"], ga["weight_decay"],
               self.fc.numel, self.fc.flat.data_ptr(), self.fc.grad.data_ptr(), ca.exp_avg.data_ptr(),
               ca.exp_avg_sq.data_ptr(), ca.step_dev.data_ptr(), ca.hyper.data_ptr(), gc["lr"], gc["betas"][0],
               gc["betas"][1], gc["eps"], gc["weight_decay"],
               100.0, self.ft.flat.data_ptr(), float(1.0 - tau), float(tau), 3, self.loss_buffer.data_ptr(),
               sq.data_ptr(), skip.data_ptr(), self._clip_scratch.data_ptr(), st)

    def soft_update_target(self, tau=0.02, skip=None):  # Agent.py:90-94
        L.require_gpu(self.fc.flat)
        L.call("dr_ema", self.fc.numel, self.ft.flat.data_ptr(), self.fc.flat.data_ptr(), float(1.0 - tau),
               float(tau), None if skip is None else skip.data_ptr(), hip.stream())

    # ---- reference API -------------------------------------------------------
    def update_S(self, lambda_returns):  # Agent.py:78-88
        R = lambda_returns.detach().float().contiguous()
        L.require_gpu(R)
        norm = torch.empty(1, device=R.device)
        L.call("dr_update_S", R.numel(), L.ptr(R), L.ptr(self.S_dev), L.ptr(norm), None, 0, hip.stream())
        return norm

    def compute_batched_R_lambda_returns(self, hidden_state_batched_seq, latent_state_batched_seq,
                                         reward_batched_seq, continue_batched_seq, seq_length):  # Agent.py:156-172
        with torch.no_grad():
            V = self.target_critic.value(hidden_state_batched_seq, latent_state_batched_seq)
            B = V.shape[0]
            H = int(seq_length)
            r = reward_batched_seq.reshape(B, H).float().contiguous()
            c = continue_batched_seq.reshape(B, H).float().contiguous()
            R = torch.empty(B, H, device=V.device)
            L.call("dr_lambda_returns", B, H, L.ptr(r), L.ptr(c), L.ptr(V.reshape(B, H + 1).contiguous()),
                   self.gamma, self.lambda_, L.ptr(R), hip.stream())
        return R.unsqueeze(-1)

    def train_step(self, z_batch_seq, h_batch_seq, reward_batch_seq, continue_batch_seq, action_batch_seq,
                   a_mu_batch_seq, a_sigma_batch_seq):
        """Agent.train_step (Agent.py:96-154) on HIP kernels.  Gradients reach
        the actor through a_mu/a_sigma's autograd graph (the HIP imagination
        unroll's backward when they come from Dreamer.dream_episodes)."""
        self._ensure_flat()
        h, z = h_batch_seq.detach().float().contiguous(), z_batch_seq.detach().float().contiguous()
        L.require_gpu(h)
        B, H1 = h.shape[:2]
        H = H1 - 1
        dev = h.device
        d = L.dr_dims()
        d.hidden, d.rows, d.cols, d.action = h.shape[-1], z[0, 0].numel(), 1, a_mu_batch_seq.shape[-1]
        d.critic_h1, d.critic_h2 = self.critic.value_net[0].out_features, self.critic.value_net[3].out_features
        d.buckets = self.buckets
        M = B * H1
        st = hip.stream()
        R = self.compute_batched_R_lambda_returns(h, z, reward_batch_seq, continue_batch_seq, H).view(B, H)
        ctape = torch.zeros(L.query("dr_critic_tape_bytes", d, M), dtype=torch.uint8, device=dev)
        V = torch.empty(B, H1, device=dev)
        L.call("dr_critic_fwd", d, self.critic_struct(), M, L.ptr(h), d.hidden, L.ptr(z), d.rows, None, L.ptr(V),
               L.ptr(ctape), None, 0, st)
        norm = self.update_S(R)
        mu = a_mu_batch_seq.detach().float().contiguous()
        sg = a_sigma_batch_seq.detach().float().contiguous()
        a = action_batch_seq.detach().float().contiguous()
        la = torch.empty(1 + B * H, device=dev)
        g_mu, g_sg = torch.empty_like(mu), torch.empty_like(sg)
        L.call("dr_actor_loss_grad", B, H, d.action, L.ptr(mu), L.ptr(sg), L.ptr(a), L.ptr(R), L.ptr(V), L.ptr(norm),
               self.nu, 1.0 / (B * H), L.ptr(la), L.ptr(g_mu), L.ptr(g_sg), st)
        ws = hip.workspace(dev).get("cbw", L.query("dr_critic_workspace_bytes", d, B, H))
        self.critic_optimiser.zero_grad()
        L.call("dr_critic_loss_bwd", d, self.critic_struct(), B, H, L.ptr(h), L.ptr(z), L.ptr(R), L.ptr(ctape),
               1.0 / (B * H), L.ptr(self.loss_slot(1)), self.critic_struct(grad=True), L.ptr(ws), ws.numel(), st)
        self.loss_slot(0).copy_(la[0:1])
        loss_actor, loss_critic = la[0].clone(), self.loss_buffer[1].clone()
        if not (torch.isfinite(loss_actor) and torch.isfinite(loss_critic)):
            print("Agent loss is nan or inf, skipping update.")
            return loss_actor, loss_critic
        self.actor_optimiser.zero_grad()
        if a_mu_batch_seq.requires_grad or a_sigma_batch_seq.requires_grad:
            torch.autograd.backward([a_mu_batch_seq, a_sigma_batch_seq], [g_mu.view_as(a_mu_batch_seq),
                                                                          g_sg.view_as(a_sigma_batch_seq)])
            self.fa.sync_grads()
        sq = torch.zeros(2, device=dev)
        skip = torch.zeros(1, dtype=torch.int32, device=dev)
        # a timed-out persistent BPTT left NaN gradients and the fault slot set
        L.call("dr_nonfinite", 1, L.ptr(self.fault_slot()), skip.data_ptr(), st)
        L.call("dr_sqnorm", self.fa.numel, self.fa.grad.data_ptr(), sq.data_ptr(), st)
        L.call("dr_sqnorm", self.fc.numel, self.fc.grad.data_ptr(), sq.data_ptr() + 4, st)
        self.critic_optimiser.fused_step(sq[1:2], 100.0, skip)
        self.actor_optimiser.fused_step(sq[0:1], 100.0, skip)
        self.soft_update_target()
        return loss_actor, loss_critic
