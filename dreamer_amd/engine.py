"""ImaginationEngine: the fused, device-resident train_Agent epoch.

One epoch (Dreamer.train_Agent's unit of work, Dreamer.py:264-287) is a fixed
sequence of libdreamer_hip calls on one stream:

  a1  window starts (host numpy RNG, Buffer.py:36-48) -> device
  a3  encoder conv stack over the S/2 warm-start frames of all B windows,
      read straight from the u8 replay ring in HBM (time-batched)
  a2  posterior scan (GRU + latent_mapper + sampler), S/2 steps
  a7  H-step imagination unroll (actor, GRU, prior, reward, continue)
  a13-a16 target/critic forward, lambda returns, update_S, actor loss and
      BPTT through the unroll, critic two-hot CE backward, clip + AdamW,
      soft target update

With world_size > 1 (one process per GPU, RCCL over xGMI) each rank runs its
slice of the batch; the exchange is one all-gather of the lambda returns
(global quantile of update_S) and one all-reduce of a flat
[actor grads | critic grads | losses] buffer.  Everything else is local.
Each phase is captured once into a HIP graph and replayed; collectives run
between the phase graphs.
"""
import contextlib
import gc

import numpy as np

import torch

from . import _lib as L
from . import hip

WARM_STREAM = 1 << 24
DREAM_STREAM = 2 << 24
_CU_STREAMS = {}  # (device index, CU mask words) -> HIP stream handle (warm_stream)


@contextlib.contextmanager
def _no_gc():
    """Stream capture with Python's cyclic collector off: an engine of an
    earlier Dreamer (they hold each other, so only the collector frees them)
    must not destroy its captured graphs while this capture is open -- a graph
    destroyed during a global-mode capture invalidates it and aborts in the
    destructor.  torch.cuda.graph collects once before capture_begin."""
    enabled = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        yield
    finally:
        if enabled:
            gc.enable()


def cu_mask_words(n_cus, fraction):
    """The 32-bit words of a CU mask keeping the first round(n_cus * fraction)
    CUs (at least one, at most all) of the device's CU-mask order."""
    keep = max(1, min(n_cus, int(round(n_cus * fraction))))
    words = [0] * ((n_cus + 31) // 32)
    for i in range(keep):
        words[i // 32] |= 1 << (i % 32)
    return words


class ImaginationEngine:
    def __init__(self, dreamer, B=None, world=None, use_graph=True):
        self.dr = dreamer
        self.dev = dreamer.device
        self.B = int(B or dreamer.batch_size)
        self.S = int(dreamer.sequence_length)
        self.H = int(dreamer.horizon)
        self.T = self.S // 2
        self.world = world  # (rank, size, group) or None
        self.rank = world[0] if world else 0
        self.wsize = world[1] if world else 1
        # the collectives run whenever a process group is given, also at size 1
        # (tests/test_gpu_rccl.py exercises the RCCL path on one GPU)
        self.dp = world is not None
        self.use_graph = use_graph
        self.graph = None
        self.graph_key = None
        # Second stream: the conv encoder of the warm start (one chunk, the
        # scan waits on it) and the critic backward beside the actor BPTT in
        # losses_and_grads(fork=True).  Measured and dropped:
        # time-chunked encoding under the posterior scan (r01 and r04:
        # slower, every later phase of the epoch 3-4x slower when fenced,
        # profiles/r04l_overlap_phase_probe.txt) and a forked critic backward
        # inside the epoch graph (~6 % slower replays, r01_ab_overlap.txt).
        self.side = torch.cuda.Stream(self.dev)
        self.chunks = [(0, self.T)]
        self._alloc()
    # ------------------------------------------------------------------ setup
    @staticmethod
    def warm_chunks(T, size=8):
        """Time chunks [t0, t1) of the warm-start window: conv chunk c+1 runs
        while the posterior scan consumes chunk c."""
        return [(t0, min(T, t0 + size)) for t0 in range(0, T, size)]

    def dims(self):
        return self.dr.world_model.dims(self.dr.agent)

    def _alloc(self):
        d = self.dims()
        self.d = d
        B, H, T = self.B, self.H, self.T
        L_ = d.rows * d.cols
        dev = self.dev
        f = lambda *s: torch.zeros(*s, device=dev)
        self.starts = torch.zeros(B, dtype=torch.int64, device=dev)
        # two pinned staging buffers; an event guards reuse (a graph replay
        # returns at once, so the next epoch's host write must not race the
        # previous epoch's pending H2D copy)
        self.starts_host = [torch.zeros(B, dtype=torch.int64).pin_memory() for _ in range(2)]
        self.copy_ev = [None, None]
        self.epochs = 0
        self.act_win = f(B, self.S, d.action)
        self.feat = f(T * B, d.enc_hidden)
        self.z0, self.h0 = f(B, L_), f(B, d.hidden)
        self.latents, self.hiddens = f(B, H + 1, L_), f(B, H + 1, d.hidden)
        self.actions, self.mus, self.sigmas = f(B, H, d.action), f(B, H, d.action), f(B, H, d.action)
        self.rewards, self.continues = f(B, H), f(B, H)
        self.V_t, self.V_c = f(B, H + 1), f(B, H + 1)
        self.R = f(B, H)
        self.R_all = f(self.wsize * B, H) if self.dp else self.R
        self.norm = f(1)
        self.loss_a = f(1 + B * H)
        self.g_mu, self.g_sig = f(B, H, d.action), f(B, H, d.action)
        self.sq = f(2)
        self.skip = torch.zeros(1, dtype=torch.int32, device=dev)
        M = B * (H + 1)
        self.ws_enc = hip.workspace(dev).get("e_enc", L.query("dr_encoder_workspace_bytes", d, T * B))
        self.ws_obs = hip.workspace(dev).get("e_obs", L.query("dr_observe_workspace_bytes", d, B))
        self.tape = torch.zeros(L.query("dr_imagine_tape_bytes", d, B, H), dtype=torch.uint8, device=dev)
        self.ws_im = hip.workspace(dev).get("e_im", L.query("dr_imagine_workspace_bytes", d, B, H))
        self.ctape = torch.zeros(L.query("dr_critic_tape_bytes", d, M), dtype=torch.uint8, device=dev)
        self.ws_cr = hip.workspace(dev).get("e_cr", L.query("dr_critic_workspace_bytes", d, B, H))
        # the online critic's forward / loss backward run on a side stream
        # beside the target critic and the BPTT (run_many): own workspace
        self.ws_cr2 = hip.workspace(dev).get("e_cr2", L.query("dr_critic_workspace_bytes", d, B, H))
        self.rng = hip.rng(dev)

    # ------------------------------------------------------------- the phases
    def encode_and_warm(self, frames, noise_q=None):
        """a3 + a2: frames is a dr_frames over (B, T) windows; actions come from
        self.act_win [B][S][A].  Writes self.z0, self.h0."""
        d, st = self.d, hip.stream()
        wm = self.dr.world_model.packed()
        L.call("dr_encoder_features", d, wm, frames, self.B, self.T, L.ptr(self.feat), L.ptr(self.ws_enc),
               self.ws_enc.numel(), st)
        if noise_q is not None:
            nz = hip.explicit_noise(q=noise_q, device=self.dev)
        else:
            nz = L.dr_noise(None, None, self.rng.state.data_ptr(), self.rank * self.B, WARM_STREAM)
        A = d.action
        L.call("dr_observe_scan", d, wm, self.B, self.T, L.ptr(self.feat), L.ptr(self.act_win), self.S * A, A, None,
               None, nz, L.ptr(self.z0), L.ptr(self.h0), None, L.ptr(self.ws_obs), self.ws_obs.numel(), st)

    def imagine(self, eps=None, q=None, deterministic=False, z0=None, h0=None, d=None):
        """a7: unroll H steps from (self.z0, self.h0) (or the given slot);
        d: dims override (the pipelined epochs pass launch_form = 1)."""
        d = self.d if d is None else d
        z0 = self.z0 if z0 is None else z0
        h0 = self.h0 if h0 is None else h0
        if eps is not None or q is not None:
            nz = hip.explicit_noise(q=q, eps=eps, device=self.dev)
        else:
            nz = L.dr_noise(None, None, self.rng.state.data_ptr(), self.rank * self.B, DREAM_STREAM)
        L.call("dr_imagine_fwd", d, self.dr.world_model.packed(), self.dr.agent.actor_struct(), self.B, self.H,
               L.ptr(z0), L.ptr(h0), nz, int(deterministic), L.ptr(self.latents), L.ptr(self.hiddens),
               L.ptr(self.actions), L.ptr(self.rewards), L.ptr(self.continues), L.ptr(self.mus),
               L.ptr(self.sigmas), L.ptr(self.tape), L.ptr(self.ws_im), self.ws_im.numel(), hip.stream())

    def returns(self):
        """target-critic values and lambda returns (Agent.py:156-172)."""
        ag, d, st = self.dr.agent, self.d, hip.stream()
        M = self.B * (self.H + 1)
        L_ = d.rows * d.cols
        L.call("dr_critic_fwd", d, ag.critic_struct(target=True), M, L.ptr(self.hiddens), d.hidden,
               L.ptr(self.latents), L_, None, L.ptr(self.V_t), None, L.ptr(self.ws_cr), self.ws_cr.numel(), st)
        L.call("dr_lambda_returns", self.B, self.H, L.ptr(self.rewards), L.ptr(self.continues), L.ptr(self.V_t),
               ag.gamma, ag.lambda_, L.ptr(self.R), st)

    def losses_and_grads(self, fork=True):
        """update_S, actor loss + BPTT, critic CE backward (Agent.py:96-145).
        With fork=True the critic backward runs on the side stream beside the
        actor's BPTT (they share only read-only inputs)."""
        ag, d = self.dr.agent, self.d
        main = torch.cuda.current_stream(self.dev)
        st = main.cuda_stream
        B, H = self.B, self.H
        M = B * (H + 1)
        L_ = d.rows * d.cols
        scale = 1.0 / float(B * self.wsize * H)
        L.call("dr_critic_fwd", d, ag.critic_struct(), M, L.ptr(self.hiddens), d.hidden, L.ptr(self.latents), L_,
               None, L.ptr(self.V_c), L.ptr(self.ctape), L.ptr(self.ws_cr), self.ws_cr.numel(), st)
        critic_args = (d, ag.critic_struct(), B, H, L.ptr(self.hiddens), L.ptr(self.latents), L.ptr(self.R),
                       L.ptr(self.ctape), scale, L.ptr(ag.loss_slot(1)), ag.critic_struct(grad=True),
                       L.ptr(self.ws_cr), self.ws_cr.numel())
        if fork:
            self.side.wait_stream(main)
            L.call("dr_critic_loss_bwd", *critic_args, self.side.cuda_stream)
        L.call("dr_update_S", self.R_all.numel(), L.ptr(self.R_all), L.ptr(ag.S_dev), L.ptr(self.norm), None, 0, st)
        L.call("dr_actor_loss_grad", B, H, d.action, L.ptr(self.mus), L.ptr(self.sigmas), L.ptr(self.actions),
               L.ptr(self.R), L.ptr(self.V_c), L.ptr(self.norm), ag.nu, scale, L.ptr(self.loss_a), L.ptr(self.g_mu),
               L.ptr(self.g_sig), st)
        if not fork:
            L.call("dr_critic_loss_bwd", *critic_args, st)
        L.call("dr_imagine_bwd", d, self.dr.world_model.packed(), ag.actor_struct(), B, H, L.ptr(self.latents),
               L.ptr(self.hiddens), L.ptr(self.actions), L.ptr(self.g_mu), L.ptr(self.g_sig), None, None, None,
               L.ptr(self.tape), ag.actor_struct(grad=True), L.ptr(self.ws_im), self.ws_im.numel(), st)
        ag.loss_slot(0).copy_(self.loss_a[0:1])
        if fork:
            main.wait_stream(self.side)

    # pieces of losses_and_grads for the two-stream update of run_many
    def _x_critic_fwd_and_prep(self):
        """side stream: online critic forward (Agent.py:105) and the BPTT's
        upstream-gradient / transposed-weight prep."""
        ag, d, st = self.dr.agent, self.d, hip.stream()
        M = self.B * (self.H + 1)
        L.call("dr_critic_fwd", d, ag.critic_struct(), M, L.ptr(self.hiddens), d.hidden, L.ptr(self.latents),
               d.rows * d.cols, None, L.ptr(self.V_c), L.ptr(self.ctape), L.ptr(self.ws_cr2), self.ws_cr2.numel(),
               st)
        L.call("dr_imagine_bwd_prep", d, self.dr.world_model.packed(), ag.actor_struct(), self.B, self.H, None,
               None, None, L.ptr(self.ws_im), self.ws_im.numel(), st)

    def _actor_loss(self):
        """update_S and the actor loss / its gradient w.r.t. mu, sigma (Agent.py:78-125)."""
        ag, d, st = self.dr.agent, self.d, hip.stream()
        B, H = self.B, self.H
        scale = 1.0 / float(B * self.wsize * H)
        L.call("dr_update_S", self.R_all.numel(), L.ptr(self.R_all), L.ptr(ag.S_dev), L.ptr(self.norm), None, 0, st)
        L.call("dr_actor_loss_grad", B, H, d.action, L.ptr(self.mus), L.ptr(self.sigmas), L.ptr(self.actions),
               L.ptr(self.R), L.ptr(self.V_c), L.ptr(self.norm), ag.nu, scale, L.ptr(self.loss_a), L.ptr(self.g_mu),
               L.ptr(self.g_sig), st)

    def _x_critic_bwd(self):
        """side stream: two-hot CE of the critic and its backward (Agent.py:127-145)."""
        ag, d = self.dr.agent, self.d
        B, H = self.B, self.H
        scale = 1.0 / float(B * self.wsize * H)
        L.call("dr_critic_loss_bwd", d, ag.critic_struct(), B, H, L.ptr(self.hiddens), L.ptr(self.latents),
               L.ptr(self.R), L.ptr(self.ctape), scale, L.ptr(ag.loss_slot(1)), ag.critic_struct(grad=True),
               L.ptr(self.ws_cr2), self.ws_cr2.numel(), hip.stream())

    def _bptt(self, d=None):
        ag, d = self.dr.agent, (self.d if d is None else d)
        L.call("dr_imagine_bwd_main", d, self.dr.world_model.packed(), ag.actor_struct(), self.B, self.H,
               L.ptr(self.latents), L.ptr(self.hiddens), L.ptr(self.actions), L.ptr(self.g_mu), L.ptr(self.g_sig),
               0, L.ptr(self.tape), ag.actor_struct(grad=True), L.ptr(self.ws_im), self.ws_im.numel(), hip.stream())
        ag.loss_slot(0).copy_(self.loss_a[0:1])

    def optimise(self):
        """non-finite skip, clip_grad_norm_(100) x2, AdamW x2, soft target (Agent.py:137-153)."""
        self.dr.agent.fused_optimiser_step(self.sq, self.skip)

    # phases of one epoch; collectives (world > 1) run between phases
    def _encode_chunk(self, t0, t1, stream_ptr):
        d = self.d
        fr = self.dr.buffer.frames_struct(self.starts)
        fr.t0 = t0
        off = t0 * self.B * d.enc_hidden * 4
        L.call("dr_encoder_features", d, self.dr.world_model.packed(), fr, self.B, t1 - t0,
               L.ptr(self.feat) + off, L.ptr(self.ws_enc), self.ws_enc.numel(), stream_ptr)

    def _scan_chunk(self, t0, t1, stream_ptr):
        """Posterior scan over window steps [t0, t1) (Dreamer.py:244-262).  A
        chunk after the first continues from (self.z0, self.h0): its first
        step runs GRU(z_{t0-1}, a_{t0-1}, h) and the sampler's Philox stream
        is offset by t0, so the draws equal the unchunked scan's."""
        d, A = self.d, self.d.action
        nz = L.dr_noise(None, None, self.rng.state.data_ptr(), self.rank * self.B, WARM_STREAM + t0)
        feat = L.ptr(self.feat) + t0 * self.B * d.enc_hidden * 4
        if t0 == 0:
            acts, zi, hi = L.ptr(self.act_win), None, None
        else:
            acts, zi, hi = L.ptr(self.act_win) + (t0 - 1) * A * 4, L.ptr(self.z0), L.ptr(self.h0)
        L.call("dr_observe_scan", d, self.dr.world_model.packed(), self.B, t1 - t0, feat, acts, self.S * A, A,
               hi, zi, nz, L.ptr(self.z0), L.ptr(self.h0), None, L.ptr(self.ws_obs), self.ws_obs.numel(),
               stream_ptr)

    def _ph_encwarm(self):
        """a3 + a2, pipelined: the conv encoder runs chunk by chunk on the side
        stream; the scan of chunk c waits only for chunk c's features."""
        main = torch.cuda.current_stream(self.dev)
        self.dr.buffer.gather_actions(self.starts, self.act_win)
        self.side.wait_stream(main)
        done = []
        with torch.cuda.stream(self.side):
            for t0, t1 in self.chunks:
                self._encode_chunk(t0, t1, self.side.cuda_stream)
                ev = torch.cuda.Event()
                ev.record(self.side)
                done.append(ev)
        for (t0, t1), ev in zip(self.chunks, done):
            main.wait_event(ev)
            self._scan_chunk(t0, t1, main.cuda_stream)

    def time_encoder(self, reps=5):
        """Average ms of the conv encoder (all chunks, back to back on one
        stream, no overlap): the dominant kernel group's live duration for the
        bench's roofline line."""
        st = torch.cuda.current_stream(self.dev)
        for t0, t1 in self.chunks:
            self._encode_chunk(t0, t1, st.cuda_stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(reps):
            for t0, t1 in self.chunks:
                self._encode_chunk(t0, t1, st.cuda_stream)
        b.record(st)
        b.synchronize()
        return a.elapsed_time(b) / reps

    def _ph_update(self):
        self.losses_and_grads(fork=False)

    def _ph_optim(self):
        self.optimise()
        L.call("dr_rng_advance", self.rng.state.data_ptr(), 1, hip.stream())

    def phases(self):
        """(name, body, collective-after) in execution order."""
        ph = [("encwarm", self._ph_encwarm, None), ("imagine", self.imagine, None),
              ("returns", self.returns, self._allgather_R if self.dp else None),
              ("update", self._ph_update, self._allreduce_grads if self.dp else None),
              ("optim", self._ph_optim, None)]
        if self.dp and not self.persistent_bptt():
            # data-parallel, BPTT in launch form: the update in two phase graphs,
            # so that the critic's gradient all-reduce (issued async on RCCL's
            # stream as soon as the critic backward is enqueued) runs under the
            # actor's BPTT; the actor part is reduced after it (Agent.py:141-148).
            # With the persistent BPTT (B <= 64 per rank) the update stays one
            # phase and the whole buffer is reduced after it: an RCCL kernel
            # holding CUs beside k_pbptt (one workgroup on every CU) could push
            # its waits past their bound
            ph[3:4] = [("critic", self._ph_critic, self._allreduce_critic_async),
                       ("actor", self._ph_actor, self._allreduce_actor)]
        return ph

    def persistent_chain(self):
        """True when the imagination unroll (and the warm start's scan) run as
        the persistent kernels: train_Agent then keeps its epochs sequential."""
        return bool(L.query("dr_persistent_kernels", self.d, self.B, self.T, self.H) & 2)

    def persistent_bptt(self):
        """True when dr_imagine_bwd runs as the one persistent k_pbptt launch."""
        return bool(L.query("dr_persistent_kernels", self.d, self.B, self.T, self.H) & 4)

    # ------------------------------------------------------- fault checks
    def check_faults(self, wait=True):
        """Raise if a persistent kernel (posterior scan, imagination unroll or
        BPTT) timed out on a wait.  Such a kernel wrote NaN over its outputs
        and the agent's fault slot, so that epoch's update was skipped on every
        rank (non-finite skip, Agent.py:137-139), and set the host-mapped fault
        word (dr_dims.fault_host), which this reads without a copy.  wait=True
        first waits for the queued work; run() / run_many() look without
        waiting, so they see a fault of an epoch that has finished.  On a
        fault: the flags are cleared, every later epoch runs the launch form
        (new graphs), and RuntimeError is raised."""
        h, _ = self.dr.agent.fault_host()
        if wait:
            torch.cuda.current_stream(self.dev).synchronize()
        if int(h[0]) != 0:
            self._on_fault()

    def _on_fault(self):
        ag = self.dr.agent
        torch.cuda.synchronize(self.dev)
        ag.fault_slot().zero_()
        ag.fault_host()[0][0] = 0
        ag.persistent_ok = False
        self.d = self.dims()
        self.graph, self.graph_key, self._pipe = None, None, None
        raise RuntimeError("dreamer_amd: a persistent kernel (posterior scan / imagination unroll / BPTT) timed out "
                           "waiting on another workgroup (not every workgroup was resident, e.g. other work held "
                           "CUs); its outputs were NaN and that epoch's actor-critic update was skipped. Every "
                           "later epoch runs the launch form.")

    def _ph_critic(self):
        """DP update, part 1: online critic forward, update_S, the actor loss
        and its dL/dmu / dL/dsigma, the critic's CE backward, both loss slots
        (the kernel order of losses_and_grads(fork=False) without the BPTT)."""
        ag, d, st = self.dr.agent, self.d, hip.stream()
        B, H = self.B, self.H
        M = B * (H + 1)
        scale = 1.0 / float(B * self.wsize * H)
        L.call("dr_critic_fwd", d, ag.critic_struct(), M, L.ptr(self.hiddens), d.hidden, L.ptr(self.latents),
               d.rows * d.cols, None, L.ptr(self.V_c), L.ptr(self.ctape), L.ptr(self.ws_cr), self.ws_cr.numel(), st)
        self._actor_loss()
        L.call("dr_critic_loss_bwd", d, ag.critic_struct(), B, H, L.ptr(self.hiddens), L.ptr(self.latents),
               L.ptr(self.R), L.ptr(self.ctape), scale, L.ptr(ag.loss_slot(1)), ag.critic_struct(grad=True),
               L.ptr(self.ws_cr), self.ws_cr.numel(), st)
        ag.loss_slot(0).copy_(self.loss_a[0:1])

    def _ph_actor(self):
        """DP update, part 2: the actor's BPTT (dr_imagine_bwd)."""
        ag, d = self.dr.agent, self.d
        L.call("dr_imagine_bwd", d, self.dr.world_model.packed(), ag.actor_struct(), self.B, self.H,
               L.ptr(self.latents), L.ptr(self.hiddens), L.ptr(self.actions), L.ptr(self.g_mu), L.ptr(self.g_sig),
               None, None, None, L.ptr(self.tape), ag.actor_struct(grad=True), L.ptr(self.ws_im), self.ws_im.numel(),
               hip.stream())

    def epoch_body(self):
        for _, body, coll in self.phases():
            body()
            if coll is not None:
                coll()

    # ------------------------------------------------------------------ DP
    def _allgather_R(self):
        import torch.distributed as dist
        parts = list(self.R_all.view(self.wsize, self.B, self.H).unbind(0))
        dist.all_gather(parts, self.R, group=self.world[2])

    def _allreduce_grads(self):
        import torch.distributed as dist
        ag = self.dr.agent
        dist.all_reduce(ag.grad_buffer, op=dist.ReduceOp.SUM, group=self.world[2])
        ag.loss_buffer.div_(self.wsize)

    def _allreduce_critic_async(self):
        """[critic grads | loss slots] of the flat buffer, async (RCCL's own
        stream waits on the current one); waited for in _allreduce_actor."""
        import torch.distributed as dist
        ag = self.dr.agent
        na = ag.fa.grad.numel()
        self._critic_work = dist.all_reduce(ag.grad_buffer[na:], op=dist.ReduceOp.SUM, group=self.world[2],
                                            async_op=True)

    def _allreduce_actor(self):
        import torch.distributed as dist
        ag = self.dr.agent
        na = ag.fa.grad.numel()
        dist.all_reduce(ag.grad_buffer[:na], op=dist.ReduceOp.SUM, group=self.world[2])
        self._critic_work.wait()
        self._critic_work = None
        ag.loss_buffer.div_(self.wsize)

    # ----------------------------------------------------------------- driver
    def run(self, starts_np, timing=False):
        """One train_Agent epoch from host window starts; returns the device
        loss slots (actor, critic).  With timing=True, HIP events bracket every
        phase (self.last_events)."""
        self.check_faults(wait=False)
        i = self.epochs & 1
        if self.copy_ev[i] is not None:
            self.copy_ev[i].synchronize()
        self.starts_host[i].copy_(torch.from_numpy(np.asarray(starts_np, dtype=np.int64)))
        self.starts.copy_(self.starts_host[i], non_blocking=True)
        self.copy_ev[i] = torch.cuda.Event()
        self.copy_ev[i].record()
        self.epochs += 1
        ag = self.dr.agent
        key = (ag.params_key(), self.dr.world_model.params_key(), self.dr.buffer.device_key())
        if self.use_graph and (self.graph is None or self.graph_key != key):
            self._capture(key)
        evs = [torch.cuda.Event(enable_timing=True)] if timing else None
        if evs:
            evs[0].record()
        for k, (name, body, coll) in enumerate(self.phases()):
            if self.use_graph:
                self.graph[k].replay()
            else:
                body()
            if coll is not None:
                coll()
            if evs:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                evs.append(e)
        self.last_events = evs
        return ag.loss_slot(0), ag.loss_slot(1)

    def phase_ms(self):
        """Per-phase milliseconds of the last timed run (after a sync)."""
        names = [p[0] for p in self.phases()]
        ev = self.last_events
        return {n: ev[k].elapsed_time(ev[k + 1]) for k, n in enumerate(names)}

    # ------------------------------------------------- pipelined epochs
    # Everything the warm start reads (world-model parameters, the replay
    # ring, the window starts, its own noise) is untouched by the actor-critic
    # update, so the warm start of epoch e+1 (conv encoder + posterior scan)
    # can run on a second stream beside the imagination / update chain of
    # epoch e.  The results are those of the sequential LAUNCH-FORM epochs bit
    # for bit (test_pipelined_epochs_match_sequential, DREAMER_PERSISTENT=0):
    # the warm start keeps its own copy of the Philox state, advanced once per
    # epoch like the main one, and (z0, h0) are double-buffered.  Every graph
    # here is captured in launch form (a persistent kernel needs every CU);
    # the sequential run() at B <= 128 uses the persistent kernels, whose
    # LayerNorm sums run in another order, so there the two agree to rounding
    # -- and Dreamer.train_Agent does not pipeline where the chain is
    # persistent (persistent_chain).
    def warm_stream(self, cu_fraction=None):
        """The stream of the pipelined warm start: a plain torch stream, or with
        cu_fraction in (0, 1) a HIP stream restricted to that share of the CUs
        (dr_stream_create_cumask) so that the imagination / update chain keeps
        CUs of its own.  DREAMER_WARM_CUS sets the default fraction (0.875:
        B = 256, K = 10 epochs, warm start fenced to 7/8 of the CUs with the
        chain at high priority 5.86 ms per epoch against 6.33 unfenced and
        6.87 sequential; fenced at normal priority 8.58, tools/pipe_probe.py,
        profiles/r04i_pipe_probe.txt)"""
        import ctypes
        import os
        if cu_fraction is None:
            cu_fraction = float(os.environ.get("DREAMER_WARM_CUS", "0.875"))
        if not 0.0 < cu_fraction < 1.0:
            return torch.cuda.Stream(self.dev)
        n = ctypes.c_int(0)
        with torch.cuda.device(self.dev):
            L.call("dr_device_cus", ctypes.byref(n))
            words = cu_mask_words(n.value, cu_fraction)
            # one masked stream per (device, mask) for the process, shared by
            # every engine: torch's allocator may still hold blocks used on it
            # after an engine is gone, so it is never destroyed mid-run
            ck = (torch.device(self.dev).index, tuple(words))
            h = _CU_STREAMS.get(ck)
            if h is None:
                mask = (ctypes.c_uint * len(words))(*words)
                h = ctypes.c_void_p()
                L.call("dr_stream_create_cumask", len(words), mask, ctypes.byref(h))
                _CU_STREAMS[ck] = h
        return torch.cuda.ExternalStream(h.value, device=self.dev)

    def _pipe_capture(self, key):
        dev, B, H = self.dev, self.B, self.H
        if getattr(self, "_pipe", None) is None:
            self._pipe = dict(
                stream=self.warm_stream(), side=torch.cuda.Stream(dev),
                rng=torch.zeros(2, dtype=torch.int64, device=dev),
                z0=[self.z0, torch.zeros_like(self.z0)],
                h0=[self.h0, torch.zeros_like(self.h0)],
                key=None)
        P = self._pipe
        if P["key"] == key:
            return P
        d, A = self.d, self.d.action
        # the warm graphs are captured here and replayed on the CU-masked warm
        # stream, the imagination and the BPTT beside them: all in launch form (a
        # persistent kernel needs every workgroup resident, which neither the
        # capture stream nor a chain sharing the CUs with the warm start can
        # vouch for)
        dw = L.dr_dims.from_buffer_copy(d)
        dw.launch_form = 1

        def warm(s):
            st = torch.cuda.current_stream(dev).cuda_stream
            self.dr.buffer.gather_actions(self.starts, self.act_win)
            self._encode_chunk(0, self.T, st)
            nz = L.dr_noise(None, None, P["rng"].data_ptr(), self.rank * B, WARM_STREAM)
            L.call("dr_observe_scan", dw, self.dr.world_model.packed(), B, self.T, L.ptr(self.feat),
                   L.ptr(self.act_win), self.S * A, A, None, None, nz, L.ptr(P["z0"][s]), L.ptr(P["h0"][s]), None,
                   L.ptr(self.ws_obs), self.ws_obs.numel(), st)
            L.call("dr_rng_advance", P["rng"].data_ptr(), 1, st)

        cs = torch.cuda.Stream(dev)
        cs.wait_stream(torch.cuda.current_stream(dev))
        graphs = {}
        with _no_gc(), torch.cuda.stream(cs):
            for s in (0, 1):
                for name, body in (("warm", lambda s=s: warm(s)),
                                   ("imagine", lambda s=s: self.imagine(z0=P["z0"][s], h0=P["h0"][s], d=dw))):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=cs):
                        body()
                    graphs[(name, s)] = g
            for name, body in (("returns", self.returns), ("xfwd", self._x_critic_fwd_and_prep),
                               ("actor_loss", self._actor_loss), ("xbwd", self._x_critic_bwd),
                               ("bptt", lambda: self._bptt(d=dw)), ("optim", self._ph_optim)):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=cs):
                    body()
                graphs[name] = g
        torch.cuda.current_stream(dev).wait_stream(cs)
        P["graphs"], P["key"] = graphs, key
        return P

    def run_many(self, starts_list):
        """len(starts_list) consecutive train_Agent epochs, pipelined (see
        above).  Returns a [K, 2] device tensor of (actor, critic) losses."""
        self.check_faults(wait=False)
        ag = self.dr.agent
        key = (ag.params_key(), self.dr.world_model.params_key(), self.dr.buffer.device_key())
        P = self._pipe_capture(key)
        G = P["graphs"]
        outer = torch.cuda.current_stream(self.dev)
        # DREAMER_CHAIN_PRIORITY (torch stream priority, -1 = high): the
        # imagination / update chain on a stream of that priority, so that its
        # latency-bound launches win CU slots over the warm start's convolutions
        # (default -1 with the fenced warm stream, 0 without: a high-priority
        # chain beside an unfenced warm stream measured 13.1 ms per epoch
        # against 6.9 sequential after sequential epochs in the same process,
        # profiles/r04n_pipe_after.txt)
        import os
        fenced = 0.0 < float(os.environ.get("DREAMER_WARM_CUS", "0.875")) < 1.0
        prio = int(os.environ.get("DREAMER_CHAIN_PRIORITY", "-1" if fenced else "0"))
        if prio != 0:
            if P.get("chain") is None or P.get("chain_prio") != prio:
                P["chain"], P["chain_prio"] = torch.cuda.Stream(self.dev, priority=prio), prio
            P["chain"].wait_stream(outer)
            with torch.cuda.stream(P["chain"]):
                losses = self._run_many(P, G, starts_list, P["chain"])
            outer.wait_stream(P["chain"])
        else:
            losses = self._run_many(P, G, starts_list, outer)
        return losses

    def _run_many(self, P, G, starts_list, main):
        import os
        K = len(starts_list)
        ag = self.dr.agent
        ws = P["stream"]
        host = torch.from_numpy(np.stack([np.asarray(x, dtype=np.int64) for x in starts_list])).pin_memory()
        losses = torch.empty(K, 2, device=self.dev)
        ws.wait_stream(main)
        with torch.cuda.stream(ws):
            dst = host.to(self.dev, non_blocking=True)
            P["rng"].copy_(self.rng.state)
        ev_w, ev_i = [None] * K, [None] * K
        # DREAMER_WARM0_MAIN: the first warm start has nothing to overlap with,
        # so it runs on the chain's stream over all CUs (the fenced stream
        # would only slow it); the later ones follow it on the fenced stream
        warm0_main = os.environ.get("DREAMER_WARM0_MAIN", "1") == "1"

        def issue_warm(e):
            s = main if (e == 0 and warm0_main) else ws
            if s is main:
                main.wait_stream(ws)  # the window starts / Philox copies above
            elif e == 1 and warm0_main:
                ws.wait_event(ev_w[0])  # warm starts share their staging buffers
            with torch.cuda.stream(s):
                if e >= 2:
                    s.wait_event(ev_i[e - 2])
                self.starts.copy_(dst[e])
                G[("warm", e & 1)].replay()
                ev_w[e] = torch.cuda.Event()
                ev_w[e].record(s)

        xs = P["side"]
        import os
        # Which update pieces run on a third stream: the online critic forward
        # + BPTT prep ("fwd", beside the target critic) and/or the critic
        # loss backward ("bwd", beside the BPTT).  Measured at B = 64
        # (bench, 30 epochs): none 242.3k, bwd 235.4k, both 228.7k, fwd
        # 224.3k steps/s -- a third stream of latency-bound launches slows
        # the critical chain more than it hides, so the default is "none".
        side = os.environ.get("DREAMER_SIDE", "none")

        def record(stream):
            ev = torch.cuda.Event()
            ev.record(stream)
            return ev

        issue_warm(0)
        for e in range(K):
            if e + 1 < K:
                issue_warm(e + 1)
            main.wait_event(ev_w[e])
            G[("imagine", e & 1)].replay()
            ev_i[e] = record(main)
            # side stream: online critic forward + BPTT prep beside the target
            # critic / lambda returns; later the critic loss backward beside
            # the actor's BPTT (they share only read-only inputs)
            s1 = xs if side in ("both", "fwd") else main
            s2 = xs if side in ("both", "bwd") else main
            if s1 is xs:
                xs.wait_event(ev_i[e])
            with torch.cuda.stream(s1):
                G["xfwd"].replay()
            ev_x1 = record(s1)
            G["returns"].replay()
            if self.dp:
                self._allgather_R()
            ev_r = record(main)
            main.wait_event(ev_x1)
            G["actor_loss"].replay()
            if s2 is xs:
                xs.wait_event(record(main) if s1 is main else ev_r)
            with torch.cuda.stream(s2):
                G["xbwd"].replay()
            ev_x2 = record(s2)
            G["bptt"].replay()
            main.wait_event(ev_x2)
            if self.dp:
                self._allreduce_grads()
            G["optim"].replay()
            losses[e].copy_(ag.loss_buffer[0:2])
        main.wait_stream(ws)
        main.wait_stream(xs)
        self.epochs += K
        self._pipe_host = host  # keep the pinned source alive until the H2D copy ran
        return losses

    def _capture(self, key):
        """Record each phase into its own HIP graph (capture does not execute;
        run() replays right after).  Collectives stay outside the graphs."""
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        graphs = []
        with _no_gc(), torch.cuda.stream(s):
            for _, body, _ in self.phases():
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    body()
                graphs.append(g)
        torch.cuda.current_stream(self.dev).wait_stream(s)
        self.graph, self.graph_key = graphs, key
