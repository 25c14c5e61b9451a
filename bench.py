"""Benchmark: imagined latent-steps/sec (B x H) of Dreamer.train_Agent epochs
on MI355X (BASELINE.json metric), 64x64x3 CarRacing-shaped synthetic replay.

  python bench.py [--gpus N --steps K --warmup W --batch B --seq S --horizon H --precision fp32|bf16]

Headline: K calls of Dreamer.train_Agent() with AC_epochs=1 at the north-star
batch (B=256 per GPU, S=64, H=15), window draws inside the timed region.
Secondaries: AC_epochs=2 (pipelined epochs), BASELINE configs[1] (B=64), the
world-model step and the full iteration.
Multi-GPU: launched by torch.distributed.run, one process per GPU; weak
scaling (B rows per GPU), RCCL all-gather of lambda returns + one all-reduce
of the flat [actor|critic|loss] gradient buffer per epoch.  Rank 0 prints ONE
JSON line.  The CPU baseline (rank 0, N=1 only) times the oracle's
reference-faithful CPU restatement on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "imagined latent-steps/sec (B×H) at 64×64 CarRacing, 1/2/4/8 MI355X"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 = f32 vector peak
# fp32 encoder convs 2-4 run f32-accurate on the bf16 MFMA with a 3-term split,
# 6 bf16 products per f32 product (conv_split.hip): their ceiling is 2500 / 6
SPLIT3_PEAK_TFLOPS = round(2500.0 / 6, 1)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)
HBM_PEAK_GBS = 8000.0
# SURVEY.md §8d figure of record: necessary dense FLOPs per imagined step at
# 64x64, S=64, H=15 (warm start 131.07 + dream 8.88 + update 11.17 MFLOP)
PATH_MFLOP_PER_STEP = {(64, 15, 64): 151.12, (50, 15, 64): 122.36, (64, 20, 128): 383.00}

CAR_RACER = dict(
    hidden_state_dims=600, latent_state_dims=[32, 32], action_dims=3, observation_dims=[64, 64],
    encoder_filter_num_1=32, encoder_filter_num_2=64, encoder_hidden_layer_nodes=200,
    decoder_filter_num_1=32, decoder_filter_num_2=64, decoder_hidden_layer_nodes=200,
    dyn_pred_hidden_num_nodes_1=200, dyn_pred_hidden_num_nodes_2=200,
    rew_pred_hidden_num_nodes_1=200, rew_pred_hidden_num_nodes_2=200,
    cont_pred_hidden_num_nodes_1=200, cont_pred_hidden_num_nodes_2=200,
    hidden_layer_actor_1_size=200, hidden_layer_actor_2_size=200,
    hidden_layer_critic_1_size=200, hidden_layer_critic_2_size=200, device="cuda",
    horizon=15, batch_size=64, nu=0.0003, lambda_=0.95, gamma=0.99, buffer_size=200000,
    sequence_length=64, seed=42, training_iterations=10000, random_iterations=500,
    actor_lr=0.00008, actor_betas=[0.9, 0.999], actor_eps=0.00001, critic_lr=0.0001,
    critic_betas=[0.9, 0.999], critic_eps=0.00001, AC_epochs=1, world_model_lr=0.0001,
    world_model_betas=[0.9, 0.999], world_model_eps=0.00001, WM_epochs=1,
    beta_prediction=1.0, beta_dynamics=0.5, beta_representation=0.1, critic_reward_buckets=255,
    env_id="CarRacing-v3",
)


def synthetic_replay(n, hw, A, seed=0):
    """u8 frames, U(-1,1) actions, N(0,1) rewards (symlog'ed as
    add_to_buffer does), continues 1 except every 1000th."""
    rng = np.random.default_rng(seed)
    frames = rng.integers(0, 256, size=(n, 3, hw[0], hw[1]), dtype=np.uint8)
    acts = rng.uniform(-1, 1, size=(n, A)).astype(np.float32)
    r = rng.standard_normal(size=(n,)).astype(np.float32)
    rews = (np.sign(r) * np.log(1.0 + np.abs(r))).astype(np.float32)
    conts = np.ones((n,), dtype=np.float32)
    conts[::1000] = 0.0
    return frames, acts, rews, conts


def encoder_flops_per_frame(c):
    """Algorithmic FLOPs of the conv stack + latent_mapper.0 feature columns
    for one frame (dense conv FLOPs; SURVEY §8d counting; encoder_depth 5 =
    configs[3]'s deeper VAE, one more 4 f2 -> 4 f2 conv)."""
    depth = int(c.get("encoder_depth", 4))
    ch = [3, c["encoder_filter_num_1"], c["encoder_filter_num_2"], 2 * c["encoder_filter_num_2"],
          4 * c["encoder_filter_num_2"]] + ([4 * c["encoder_filter_num_2"]] if depth == 5 else [])
    h, w = c["observation_dims"]
    fl = 0
    for i in range(depth):
        h, w = h // 2, w // 2
        fl += 2 * h * w * ch[i + 1] * ch[i] * 16
    F = ch[depth] * h * w
    return fl + 2 * F * c["encoder_hidden_layer_nodes"]


def path_mflop_per_step(c, S, H):
    """SURVEY §8d necessary MFLOP per imagined step; for the deeper VAE the
    4-conv figure of the same resolution plus the encoder's per-frame delta
    over the S/2 warm-start frames of each window (per imagined step: x S/2 / H)."""
    res = c["observation_dims"][0]
    base = PATH_MFLOP_PER_STEP.get((S, H, res))
    if base is None or int(c.get("encoder_depth", 4)) == 4:
        return base
    c4 = dict(c, encoder_depth=4)
    return round(base + (encoder_flops_per_frame(c) - encoder_flops_per_frame(c4)) / 1e6 * (S // 2) / H, 2)


def wm_step_flops(c, B, T):
    """Algorithmic (dense) FLOPs of one WorldModel.training_step on B windows
    of T steps: encoder on all B*T frames, posterior scan, prior / reward /
    continue heads and decoder on the B*(T-1) rows the losses read
    (WorldModel.py:141-145), backward = 2x forward minus the first conv's
    (unneeded) input gradient."""
    Hd, (R, C), A = c["hidden_state_dims"], c["latent_state_dims"], c["action_dims"]
    L = R * C
    eh, dh = c["encoder_hidden_layer_nodes"], c["decoder_hidden_layer_nodes"]
    h, w = c["observation_dims"]
    M, M1 = B * T, B * (T - 1)
    f1, f2 = c["decoder_filter_num_1"], c["decoder_filter_num_2"]
    conv1 = 2 * (h // 2) * (w // 2) * c["encoder_filter_num_1"] * 3 * 16
    enc = encoder_flops_per_frame(c) * M
    scan = M * 2 * (3 * Hd * (L + A + Hd) + eh * Hd + L * eh)
    p1, p2 = c["dyn_pred_hidden_num_nodes_1"], c["dyn_pred_hidden_num_nodes_2"]
    r1, r2 = c["rew_pred_hidden_num_nodes_1"], c["rew_pred_hidden_num_nodes_2"]
    q1, q2 = c["cont_pred_hidden_num_nodes_1"], c["cont_pred_hidden_num_nodes_2"]
    nb = c["critic_reward_buckets"]
    Fd = 4 * f2 * (h // 16) * (w // 16)
    heads = 2 * (Hd * p1 + p1 * p2 + p2 * L + (Hd + L) * r1 + r1 * r2 + r2 * nb + (Hd + L) * q1 + q1 * q2 + q2
                 + (Hd + L) * dh + dh * Fd)
    chans = [4 * f2, 2 * f2, f2, f1, 3]
    dec = 0
    hh, ww = h // 16, w // 16
    for i in range(4):
        dec += 2 * hh * ww * chans[i] * chans[i + 1] * 16
        hh, ww = 2 * hh, 2 * ww
    fwd = enc + scan + M1 * (heads + dec)
    return 3 * fwd - conv1 * M


def bench_wm(d, B, steps, warmup):
    """WorldModel.training_step throughput (sequences/s) fed from the device
    replay ring (Dreamer.train_world_model's unit of work)."""
    wm = d.world_model
    for _ in range(warmup):
        wm.train_step_ring(d.buffer, d.buffer.sample_start_indices(B))
    torch.cuda.synchronize()
    st = [d.buffer.sample_start_indices(B) for _ in range(steps)]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for s in st:
        wm.train_step_ring(d.buffer, s)
    ev1.record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return el / steps, ev0.elapsed_time(ev1) / 1e3 / steps, float(wm.last_losses[0])


def bench_acting(d, dev, n=100):
    """Device work of one env step of rollout_policy / evaluate_agent / Run
    (Dreamer.py:177-226, 295-322): the fused dr_act_step launch vs the unfused
    observe_step + Actor.act calls it replaces (host wall, frame H2D included)."""
    g = np.random.default_rng(7)
    frames = [g.integers(0, 256, size=(64, 64, 3), dtype=np.uint8) for _ in range(4)]
    with torch.no_grad():
        a, _, _, z, h = d.act_step(frames[0])

        def unfused(i):
            _, ot = d._obs_tensor(frames[i % 4])
            z2, h2, _ = d.world_model.observe_step(z, h, a, ot)
            d.agent.actor.act(h2, z2, deterministic=True)

        def fused(i):
            d.act_step(frames[i % 4], z, h, a, deterministic=True)

        out = {}
        for name, fn in (("unfused_us", unfused), ("fused_us", fused)):
            for i in range(5):
                fn(i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(n):
                fn(i)
            torch.cuda.synchronize()
            out[name] = round((time.perf_counter() - t0) / n * 1e6, 1)
    ts = d._act_bufs["ws"][0:128].view(torch.int64).cpu()
    out["fused_kernel_us"] = round(float(ts[15] - ts[0]) / 100.0, 1)
    out["note"] = ("per env step, batch 1: dr_act_step = GRU + conv encoder + sampler + actor in one launch "
                   "(XCD-hierarchical grid barrier); fused_kernel_us from the kernel's own clock")
    return out


def cpu_info():
    """CPU model and core counts of this host (for the cpu_baseline record)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        import psutil
        phys = psutil.cpu_count(logical=False)
    except Exception:
        phys = None
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    return model, phys, affinity


def cgroup_cpus():
    """CPUs this process may keep busy under its cgroup quota (v2 cpu.max or
    v1 cfs quota / period); None when unlimited or unreadable."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, q // per)
    except (OSError, ValueError):
        return None


class CpuEpoch:
    """Reference-faithful CPU train_Agent epoch (the oracle restatement of
    Dreamer.train_Agent, Dreamer.py:264-287): warm start with the un-detached
    graph, dream, train_step with the backward into everything (warm start
    included), two clip_grad_norm_ + AdamW steps, EMA target.  The same op
    sequence as the reference; tools/cpu_fidelity.py times it against the
    imported reference in the build container (profiles/r02_cpu_fidelity.json)."""

    def __init__(self, cfg, B, S, H, seed=0):
        from oracle import dreamer_oracle as O
        from dreamer_amd import Dreamer
        self.O = O
        c = dict(cfg)
        c.update(device="cpu", batch_size=B, sequence_length=S, horizon=H)
        torch.manual_seed(seed)
        d = Dreamer(c, torch.device("cpu"))
        self.P = {k: v.detach().clone().requires_grad_(v.dtype == torch.float32 and "buckets" not in k)
                  for k, v in d.state_dict().items()}
        self.R, self.C = c["latent_state_dims"]
        self.A = c["action_dims"]
        self.B, self.S, self.H = B, S, H
        self.frames, self.acts, _, _ = synthetic_replay(max(4096, 8 * S), c["observation_dims"], self.A, seed=0)
        self.rng = np.random.default_rng(1)
        self.actor = [self.P["agent." + k] for k in O.ACTOR_KEYS]
        self.critic = [self.P["agent." + k] for k in O.CRITIC_KEYS]
        self.m = {id(p): (torch.zeros_like(p), torch.zeros_like(p)) for p in self.actor + self.critic}
        self.S_val = 1.0
        self.step = 0

    def set_inputs(self, obs, act, q_warm, eps, q):
        """Feed explicit inputs/noise for the next epoch (fidelity timing)."""
        self._fixed = (obs, act, q_warm, eps, q)

    def epoch(self):
        O, B, S, H, R, C, A = self.O, self.B, self.S, self.H, self.R, self.C, self.A
        self.step += 1
        fixed = getattr(self, "_fixed", None)
        if fixed is None:
            st = self.rng.integers(0, len(self.frames) - S, size=B)
            idx = st[:, None] + np.arange(S)[None, :]
            obs = torch.tensor(self.frames[idx], dtype=torch.float32)
            act = torch.tensor(self.acts[idx])
            qw = torch.empty(S // 2, B * R, C).exponential_()
            eps = torch.randn(H, B, 1, A)
            q = torch.empty(H, B * R, C).exponential_()
        else:
            obs, act, qw, eps, q = fixed
        z0, h0 = O.warm_start(obs, act, S, self.P, qw, R, C)
        z, h, a, r, cc, mu, sg = O.dream(z0, h0, self.P, eps, q, H, R, C)
        la, lc, Rl, self.S_val = O.ac_losses(z, h, r, cc, a, mu, sg, self.P, self.S_val)
        for p in self.actor + self.critic:
            p.grad = None
        lc.backward()
        la.backward()  # traverses the dream AND the warm-start graph, as the reference does
        for ps, lr in ((self.critic, 1e-4), (self.actor, 8e-5)):
            gs, _ = O.clip_grad_norm([p.grad for p in ps])
            with torch.no_grad():
                for p, g in zip(ps, gs):
                    mm, vv = self.m[id(p)]
                    pn, mn, vn = O.adamw_step(p, g, mm, vv, self.step, lr)
                    p.copy_(pn); mm.copy_(mn); vv.copy_(vn)
        with torch.no_grad():
            for k in O.CRITIC_KEYS:
                t = self.P["agent.target_" + k]
                t.mul_(0.98).add_(0.02 * self.P["agent." + k])
        return float(la), float(lc)


def cpu_epoch_rates(ce, B, H, budget_s, threads):
    """Three timed samples of the CPU epoch on `threads` threads (each >= one
    epoch, stopping once a sample passes budget_s / 3), sorted."""
    torch.set_num_threads(threads)
    ce.epoch()  # warm-up at this thread count (not timed)
    rates = []
    for _ in range(3):
        n, t0 = 0, time.perf_counter()
        while True:
            ce.epoch()
            n += 1
            el = time.perf_counter() - t0
            if el >= budget_s / 3 or n >= 20:
                break
        rates.append(B * H * n / el)
    return sorted(rates)


def cpu_baseline(cfg, B, S, H, budget_s=30.0, threads=None):
    """The reference-faithful CPU epoch timed on the host's physical cores
    (SURVEY §8d), capped by the CPUs this process may use (affinity, cgroup
    quota); median of three samples.  The 16-thread rate of earlier rounds is
    kept as an extra field when the core count differs."""
    model, phys, affinity = cpu_info()
    quota = cgroup_cpus()
    usable = min(x for x in (phys, affinity, quota) if x) if (phys or affinity or quota) else 1
    threads = threads or usable
    ce = CpuEpoch(cfg, B, S, H)
    rates = cpu_epoch_rates(ce, B, H, budget_s, threads)
    res = dict(value=round(rates[1], 1), unit="imagined latent-steps/s", cores=threads, kind="port",
               min_of_3=round(rates[0], 1), median_of_3=round(rates[1], 1), max_of_3=round(rates[2], 1),
               cpu_model=model, physical_cores_host=phys, cpus_available=affinity, cgroup_cpu_quota=quota,
               fidelity="profiles/r02_cpu_fidelity.json (oracle reference-faithful epoch vs the imported "
                        "reference, same inputs, build container)",
               sample=f"3 samples of >= 1 reference-faithful train_Agent epoch (oracle CPU restatement, fp32, "
                      f"warm-start backward included) at B={B} S={S} H={H} "
                      f"{cfg['observation_dims'][0]}x{cfg['observation_dims'][1]}x3 on {threads} threads "
                      f"(min of physical cores, affinity, cgroup quota); value = median")
    if threads != 16 and usable >= 16:
        r16 = cpu_epoch_rates(ce, B, H, budget_s, 16)
        res["threads16"] = {"value": round(r16[1], 1), "min_of_3": round(r16[0], 1), "max_of_3": round(r16[2], 1)}
    return res


def traffic_for(B, res, precision):
    """HBM-side bytes of the encoder group per epoch measured by
    tools/pmc_traffic.sh for this workload (profiles/r02_traffic_*.json)."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", f"r0*_traffic_B{B}_r{res}_{precision}.json")))
    if not paths:
        return None, None
    path = paths[-1]  # the latest round's measurement of the shipped kernels
    t = json.load(open(path))
    return t.get("encoder_bytes_per_epoch"), os.path.relpath(path, REPO)


def profile_encoder_ms(precision):
    """Encoder-group kernel time per epoch from the latest committed rocprofv3
    --kernel-trace --stats summary of the headline bench command
    (profiles/r*_kernel_stats*.txt; tools/prof_summary.py format): the sum of
    the average durations of every kernel launched as often as the fused conv1 +
    conv2 kernel (one launch per encode: the convs, their weight repacks, the
    projection).  Returns (ms, kernels, source, source_hash or None) or Nones."""
    import glob
    import re
    tag = "_bf16" if precision == "bf16" else ""
    paths = [p for p in sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_kernel_stats{tag}.txt")))
             if precision == "bf16" or "_bf16" not in p]
    if not paths:
        return None, None, None, None
    path = paths[-1]
    rows = []
    src = None
    for line in open(path):
        if line.startswith("# source "):
            src = line.split()[2]
        m = re.match(r"\s*([\d.]+)\s+(\d+)\s+([\d.]+)\s+(.*)", line)
        if m:
            rows.append((int(m.group(2)), float(m.group(3)), m.group(4)))
    enc = [r for r in rows if "k_enc12" in r[2]]
    if not enc:
        return None, None, None, None
    n = enc[0][0]
    grp = [r for r in rows if r[0] == n]
    return sum(r[1] for r in grp) / 1e3, [r[2].split("(")[0][:60] for r in grp], os.path.relpath(path, REPO), src


def make_dreamer(cfg, dev, B, S, H, res, ac_epochs, world, rank, group, precision, depth=4):
    from dreamer_amd import Dreamer
    from dreamer_amd.engine import ImaginationEngine
    c = dict(cfg)
    c.update(batch_size=B, sequence_length=S, horizon=H, observation_dims=[res, res], AC_epochs=ac_epochs,
             buffer_size=max(4096, 8 * S) if res <= 64 else max(1024, 8 * S), precision=precision,
             encoder_depth=depth)
    torch.manual_seed(0)
    d = Dreamer(c, dev)
    fr, ac, rw, ct = synthetic_replay(c["buffer_size"], c["observation_dims"], c["action_dims"], seed=0)
    d.buffer.load_arrays(fr, ac, rw, ct)
    d.buffer._mirror()
    if world > 1:
        d.world = (rank, world, group)
        d.world_model.set_data_parallel(rank, world, group)
    d._engine = ImaginationEngine(d, B=B, world=(rank, world, group) if world > 1 else None)
    return c, d


VEC_OBS_DIM = 24  # configs[4] proprioceptive vector observations (a walker-like state size)


def make_vector_dreamer(cfg, dev, B, S, H, world, rank, group):
    """BASELINE configs[4]: vector observations (observation_dims=[D], MLP
    encoder / decoder, include/dreamer_hip.h dr_dims.obs_dim), synthetic f32
    replay (N(0,1) observations, U(-1,1) actions, symlog N(0,1) rewards)."""
    from dreamer_amd import Dreamer
    from dreamer_amd.engine import ImaginationEngine
    c = dict(cfg)
    n = max(8192, 8 * S)
    c.update(batch_size=B, sequence_length=S, horizon=H, observation_dims=[VEC_OBS_DIM], AC_epochs=1, buffer_size=n)
    torch.manual_seed(0)
    d = Dreamer(c, dev)
    rng = np.random.default_rng(0)
    rew = rng.standard_normal(n).astype(np.float32)
    d.buffer.load_arrays(rng.standard_normal((n, VEC_OBS_DIM)).astype(np.float32),
                         rng.uniform(-1, 1, (n, c["action_dims"])).astype(np.float32),
                         np.sign(rew) * np.log1p(np.abs(rew)), np.ones(n, np.float32))
    d.buffer._mirror()
    if world > 1:
        d.world = (rank, world, group)
        d.world_model.set_data_parallel(rank, world, group)
    d._engine = ImaginationEngine(d, B=B, world=(rank, world, group) if world > 1 else None)
    return c, d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="timed train_Agent() calls")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="imagination rows per GPU (north star: 256)")
    ap.add_argument("--seq", type=int, default=64)
    ap.add_argument("--horizon", type=int, default=15)
    ap.add_argument("--res", type=int, default=64,
                    help="frame side (64: CarRacing; 128: configs[3]'s frames with the reference's 4-conv encoder)")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                    help="fp32: parity mode (bit-exact indices vs the reference); bf16: perf mode")
    ap.add_argument("--cpu-budget", type=float, default=24.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="headline only")
    ap.add_argument("--wm-steps", type=int, default=10, help="world-model training steps timed (0: skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("DREAMER_DIST_BACKEND") == "gloo":
        local %= max(1, torch.cuda.device_count())  # rehearsal: several ranks may share one GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        import torch.distributed as dist
        # nccl = RCCL over xGMI; DREAMER_DIST_BACKEND=gloo rehearses N ranks on one GPU
        backend = os.environ.get("DREAMER_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
        group = dist.group.WORLD

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor([x], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t)
        return x

    def time_train_agent(d, steps, warmup):
        """K calls of Dreamer.train_Agent() (Dreamer.py:264-287) after W
        untimed ones.  Each call draws its window starts (np.random, the
        reference's Buffer sampling) inside the timed region."""
        for _ in range(warmup):
            d.train_Agent()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            la, lc = d.train_Agent()
        barrier()
        return max_over_ranks(time.perf_counter() - t0), (float(la), float(lc))

    B, S, H, res = args.batch, args.seq, args.horizon, args.res
    np.random.seed(1000 + rank)
    cfg, d = make_dreamer(CAR_RACER, dev, B, S, H, res, 1, world, rank, group, args.precision)
    el, (la, lc) = time_train_agent(d, args.steps, args.warmup)
    value = world * B * H * args.steps / el
    eng = d._engine
    frames = B * (S // 2)
    enc_flops = encoder_flops_per_frame(cfg) * frames
    secondary = {}
    if not args.no_secondary:
        # AC_epochs = 2 (car_racer_config.yaml): the warm start of epoch e+1 overlaps epoch e's update
        d.AC_epochs, d.pipeline_epochs = 2, True
        el2, _ = time_train_agent(d, max(2, args.steps // 2), 2)
        # the same schedule over 10 epochs per call (one warm start exposed per call instead of one in two)
        d.AC_epochs = 10
        el10, _ = time_train_agent(d, 2, 1)
        d.AC_epochs, d.pipeline_epochs = 1, False
        secondary["ac_epochs2_pipelined"] = {
            "value": round(world * B * H * 2 * max(2, args.steps // 2) / el2, 1), "unit": "imagined latent-steps/s",
            "ms_per_epoch": round(el2 / (2 * max(2, args.steps // 2)) * 1e3, 4),
            "vs_sequential": round((el / args.steps) / (el2 / (2 * max(2, args.steps // 2))), 4),
            "ac_epochs10": {"value": round(world * B * H * 10 * 2 / el10, 1),
                            "ms_per_epoch": round(el10 / 20 * 1e3, 4),
                            "vs_sequential": round((el / args.steps) / (el10 / 20), 4)},
            "note": "Dreamer.train_Agent() with AC_epochs=2 (and 10) and the pipeline_epochs config key (on by "
                    "default): the warm start of epoch e+1 on a stream fenced to 7/8 of the CUs beside epoch e's "
                    "update on a high-priority stream, the first warm start of a call on the chain stream (equal "
                    "to the sequential epochs in tests/test_gpu_parity.py; DESIGN.md 5a)"}
        if (B, S, H, res) != (64, 64, 15, 64):
            _, d64 = make_dreamer(CAR_RACER, dev, 64, 64, 15, 64, 1, world, rank, group, args.precision)
            el64, _ = time_train_agent(d64, args.steps, args.warmup)
            secondary["configs1_B64"] = {
                "value": round(world * 64 * 15 * args.steps / el64, 1), "unit": "imagined latent-steps/s",
                "ms_per_epoch": round(el64 / args.steps * 1e3, 4),
                "note": "BASELINE configs[1] shape (B=64/GPU S=64 H=15), Dreamer.train_Agent() AC_epochs=1"}
            # the reference's default AC_epochs = 2 (car_racer_config.yaml:44) at configs[1]'s B = 64: the
            # default train_Agent (sequential epochs on the persistent kernels) against the pipelined schedule
            # (engine.run_many: warm start of epoch e+1 beside epoch e, everything in launch form)
            k2 = max(2, args.steps // 2)
            d64.AC_epochs, d64.pipeline_epochs = 2, True
            el_seq, _ = time_train_agent(d64, k2, 2)

            def pipelined_calls(dd, k, w):
                e = dd._engine
                for i in range(w + k):
                    if i == w:
                        barrier()
                        t0 = time.perf_counter()
                    e.run_many([dd.buffer.sample_start_indices(64) for _ in range(2)])
                barrier()
                return max_over_ranks(time.perf_counter() - t0)
            el_pipe = pipelined_calls(d64, k2, 2)
            secondary["configs1_B64_ac_epochs2"] = {
                "value": round(world * 64 * 15 * 2 * k2 / el_seq, 1), "unit": "imagined latent-steps/s",
                "ms_per_epoch": round(el_seq / (2 * k2) * 1e3, 4),
                "pipelined_launch_form": {"value": round(world * 64 * 15 * 2 * k2 / el_pipe, 1),
                                          "ms_per_epoch": round(el_pipe / (2 * k2) * 1e3, 4)},
                "note": "configs[1] shape with the reference's AC_epochs=2: value = Dreamer.train_Agent() as shipped "
                        "(B <= 128: sequential epochs on the persistent scan / unroll / BPTT); pipelined_launch_form "
                        "= the same epochs through engine.run_many (DESIGN.md 5a)"}
            del d64
        if args.precision == "fp32":
            # bf16 perf mode (config key precision="bf16"; BASELINE configs[1] names bf16):
            # the encoder's convolutions and feature projection on the bf16 MFMA
            bf = {}
            # B = 64 first: the bf16 WM step timed with the B = 256 model (below) left the
            # B = 64 epochs measured after it ~9 % slower in the same process (r04e vs r04o)
            for tag, bb in (("configs1_B64", 64), ("north_star_B256", B)):
                if tag == "configs1_B64" and bb == B:
                    continue
                cb, db = make_dreamer(CAR_RACER, dev, bb, S, H, res, 1, world, rank, group, "bf16")
                elb, (lab, lcb) = time_train_agent(db, args.steps, args.warmup)
                enc_b = db._engine.time_encoder(reps=5) / 1e3
                fl_b = encoder_flops_per_frame(cb) * bb * (S // 2)
                ach = fl_b / enc_b / 1e12
                bf[tag] = {"value": round(world * bb * H * args.steps / elb, 1), "unit": "imagined latent-steps/s",
                           "ms_per_epoch": round(elb / args.steps * 1e3, 4), "dtype": "bf16", "B_per_gpu": bb,
                           "losses": {"actor": lab, "critic": lcb},
                           "roofline": {"bound": "mfma", "kernel": "encoder conv stack + feature projection",
                                        "achieved": round(ach, 2), "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                                        "frac": round(ach / BF16_MFMA_PEAK_TFLOPS, 4),
                                        "encoder_ms": round(enc_b * 1e3, 4)}}
                if tag == "north_star_B256" and args.wm_steps > 0:
                    # WorldModel.training_step in bf16 mode: the convolutions (encoder, decoder, their data and
                    # weight gradients) as one-term bf16 implicit GEMMs (tests/test_gpu_wm.py states the bounds)
                    wb_s, wb_gpu_s, wb_loss = bench_wm(db, bb, args.wm_steps, 2)
                    wb_s, wb_gpu_s = max_over_ranks(wb_s), max_over_ranks(wb_gpu_s)
                    bf[tag]["wm_step"] = {"value": round(world * bb / wb_s, 1), "unit": "sequences/s",
                                          "ms_per_step": round(wb_s * 1e3, 3),
                                          "gpu_ms_per_step": round(wb_gpu_s * 1e3, 3), "loss": wb_loss, "T": H}
                del db
            bf["note"] = ("Dreamer(config with precision='bf16'): conv1+conv2 fused from the u8 ring, conv3/conv4 "
                          "and the projection as bf16 implicit GEMMs (f32 accumulate); in the imagination / update "
                          "chain the GEMM-shaped products (GRU hidden product, prior / actor / heads, BPTT input "
                          "gradients, actor / critic weight gradients) take one-term bf16 operands with f32 "
                          "accumulation, while the samplers, gates, LayerNorms, optimiser and losses stay f32 "
                          "(INTEGRATION.md; tests/test_gpu_bf16.py states the tolerances)")
            secondary["bf16_perf_mode"] = bf
        # BASELINE configs[3]: 128x128 frames, the deeper VAE (encoder_depth = 5), H = 20, S = 64 at its
        # per-GPU share of the global batch 256 over 8 GPUs (B = 32) and at the whole batch on one GPU
        c3 = {}
        for bb in (32, 256):
            cc, dc = make_dreamer(CAR_RACER, dev, bb, 64, 20, 128, 1, world, rank, group, "fp32", depth=5)
            k3 = max(3, args.steps // 2)
            el3, (la3, lc3) = time_train_agent(dc, k3, 2)
            v3 = world * bb * 20 * k3 / el3
            mf3 = path_mflop_per_step(cc, 64, 20)
            enc3 = dc._engine.time_encoder(reps=3) / 1e3
            fl3 = encoder_flops_per_frame(cc) * bb * 32
            c3[f"B{bb}"] = {"value": round(v3, 1), "unit": "imagined latent-steps/s",
                            "ms_per_epoch": round(el3 / k3 * 1e3, 4), "B_per_gpu": bb, "dtype": "f32",
                            "losses": {"actor": la3, "critic": lc3},
                            "path_roofline": {"mflop_per_imagined_step": mf3,
                                              "achieved": round(v3 * mf3 * 1e6 / 1e12, 2),
                                              "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                                              "frac": round(v3 * mf3 * 1e6 / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)},
                            "encoder": {"ms": round(enc3 * 1e3, 4), "tflops": round(fl3 / enc3 / 1e12, 2),
                                        "gflop": round(fl3 / 1e9, 2)}}
            del dc
        c3["note"] = ("BASELINE configs[3] (128x128 frames, deeper VAE, S=64, H=20; global B=256 on 8 GPUs = 32 per "
                      "GPU): Dreamer.train_Agent() AC_epochs=1 with encoder_depth=5 (one more k4 s2 conv each way, "
                      "the framework's definition: the reference has no deeper VAE); fp32 mode")
        c3["parity"] = ("unpinned against the reference (framework-defined architecture): checked only against the "
                        "oracle's restatement of the same definition (tests/test_gpu_deep_vae.py)")
        secondary["configs3_deep_vae_128px_H20"] = c3
        # BASELINE configs[4]: vector observations, B = 4096 H = 15 (S = 64 assumed)
        _, dv = make_vector_dreamer(CAR_RACER, dev, 4096, 64, 15, world, rank, group)
        kv = max(3, args.steps // 4)
        elv, (lav, lcv) = time_train_agent(dv, kv, 2)
        secondary["configs4_vector_B4096"] = {
            "value": round(world * 4096 * 15 * kv / elv, 1), "unit": "imagined latent-steps/s",
            "ms_per_epoch": round(elv / kv * 1e3, 4), "dtype": "f32", "obs_dim": VEC_OBS_DIM,
            "losses": {"actor": lav, "critic": lcv},
            "note": "BASELINE configs[4] (B=4096/GPU, H=15, S=64): observation_dims=[24], MLP encoder instead of "
                    "the conv stack (no reference counterpart), Dreamer.train_Agent() AC_epochs=1",
            "parity": "unpinned against the reference (framework-defined MLP encoder): checked only against the "
                      "oracle's restatement (tests/test_gpu_vector.py)"}
        del dv
    wm = None
    if args.wm_steps > 0:
        wm_s, wm_gpu_s, wm_loss = bench_wm(d, B, args.wm_steps, 2)
        wm = (max_over_ranks(wm_s), max_over_ranks(wm_gpu_s), wm_loss)
    if rank != 0:
        barrier()
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    # the dominant kernel group (conv encoder + feature projection) timed live
    # with HIP events on the engine's stream, back to back, after the timed region
    enc_s = eng.time_encoder(reps=5) / 1e3
    peak = BF16_MFMA_PEAK_TFLOPS if args.precision == "bf16" else SPLIT3_PEAK_TFLOPS
    path_peak = BF16_MFMA_PEAK_TFLOPS if args.precision == "bf16" else FP32_MFMA_PEAK_TFLOPS
    achieved = enc_flops / enc_s / 1e12
    traffic, traffic_src = traffic_for(B, res, args.precision)
    dtype = "bf16" if args.precision == "bf16" else "f32"
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "imagined latent-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": dtype,
        "data": "synthetic (SURVEY §8d replay: u8 uniform frames, U(-1,1) actions, symlog N(0,1) rewards); "
                "reference default init under torch.manual_seed(0)",
        "config": {"workload": f"Dreamer.train_Agent() with AC_epochs=1 (replay sample + warm start S/2 + "
                               f"H-step imagination + actor-critic update), B={B}/GPU S={S} H={H} {res}x{res}x3, "
                               f"precision={args.precision}"
                               + (" (north-star batch per GPU)" if (B, S, H, res) == (256, 64, 15, 64) else ""),
                   "global_batch": B * world, "seq_len": S, "horizon": H, "parallelism": f"dp{world}",
                   "precision": args.precision},
        "roofline": {"bound": "mfma", "kernel": "encoder conv stack + feature projection (one train_Agent epoch's "
                                                 f"{frames} warm-start frames)",
                     "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": traffic,
                     "traffic_unit": "HBM-side bytes per launch group (per epoch)", "traffic_source": traffic_src,
                     "algorithmic_flops_per_launch": enc_flops,
                     "algorithmic_unit": "55.77 MFLOP per 64x64 frame (SURVEY §8d) x B*S/2 frames",
                     "encoder_ms": round(enc_s * 1e3, 4),
                     "peak_note": ("bf16 MFMA dense peak" if args.precision == "bf16" else
                                   "f32 work on the bf16 MFMA, 6 split products per f32 product (2500/6); "
                                   "the f32-input MFMA peak is 157.3 (frac_vs_f32_mfma_peak), the bf16 pipe the "
                                   "split products occupy 2500 (frac_vs_bf16_pipe)")},
        "losses": {"actor": la, "critic": lc},
    }
    if args.precision != "bf16":
        out["roofline"]["frac_vs_f32_mfma_peak"] = round(achieved / FP32_MFMA_PEAK_TFLOPS, 4)
        out["roofline"]["frac_vs_bf16_pipe"] = round(6 * achieved / BF16_MFMA_PEAK_TFLOPS, 4)
    if (B, S, H, res) == (256, 64, 15, 64):
        # the same group from the committed kernel trace (per-kernel averages under the profiler)
        pms, pk, psrc, phash = profile_encoder_ms(args.precision)
        if pms:
            sys.path.insert(0, os.path.join(REPO, "tools"))
            from prof_summary import source_hash
            same = phash is not None and phash == source_hash()
            out["roofline"]["profile"] = {"encoder_ms": round(pms, 4), "frac": round(enc_flops / (pms / 1e3) / 1e12 / peak, 4),
                                          "live_over_profile": round(enc_s * 1e3 / pms, 4), "kernels": pk,
                                          "source": psrc, "source_hash": phash, "matches_tree": same,
                                          "note": ("committed kernel trace of this source tree" if same else
                                                   "HISTORICAL: committed kernel trace of another source tree")}
    mf = PATH_MFLOP_PER_STEP.get((S, H, res))
    if mf is not None:
        tf = value * mf * 1e6 / 1e12
        out["path_roofline"] = {"bound": "mfma", "achieved": round(tf, 2), "peak": path_peak,
                                "unit": "TFLOP/s", "frac": round(tf / path_peak, 4),
                                "mflop_per_imagined_step": mf,
                                "note": "whole train_Agent epoch, SURVEY §8d necessary FLOPs x imagined steps/s"}
        # the chain: everything but the encoder group (warm-start scan, dream, update) per epoch
        chain_fl = mf * 1e6 * B * H - enc_flops
        chain_s = el / args.steps - enc_s
        if chain_s > 0:
            ctf = chain_fl / chain_s / 1e12
            out["chain_roofline"] = {"bound": "mfma", "achieved": round(ctf, 2), "peak": path_peak, "unit": "TFLOP/s",
                                     "frac": round(ctf / path_peak, 4), "gflop_per_epoch": round(chain_fl / 1e9, 2),
                                     "ms_per_epoch": round(chain_s * 1e3, 4),
                                     "note": "non-encoder FLOPs of the epoch (SURVEY §8d total - encoder group) over "
                                             "the epoch time minus the live encoder time"}
    if wm is not None:
        wm_s, wm_gpu_s, wm_loss = wm
        fl = wm_step_flops(cfg, B, H)
        ac_s = el / args.steps
        secondary["wm_step"] = {
            "value": round(world * B / wm_s, 1), "unit": "sequences/s", "ms_per_step": round(wm_s * 1e3, 3),
            "gpu_ms_per_step": round(wm_gpu_s * 1e3, 3), "B_per_gpu": B, "T": H, "loss": wm_loss,
            "mfma_tflops": round(fl / wm_s / 1e12, 2), "mfma_frac_f32": round(fl / wm_s / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4),
            "algorithmic_gflop": round(fl / 1e9, 2),
            "note": "WorldModel.training_step (posterior scan, decoder, losses, full backward, clip, AdamW) from the "
                    "device replay ring; under DP the mask / loss sums and the flat gradient are all-reduced (RCCL)"}
        secondary["full_iteration"] = {
            "value": round(world * B * H / (wm_s + ac_s), 1), "unit": "imagined latent-steps/s",
            "ms_per_iteration": round((wm_s + ac_s) * 1e3, 3),
            "note": "1 WM step + 1 train_Agent epoch per iteration (WM_epochs = AC_epochs = 1)"}
    if not args.no_secondary and res == 64:
        secondary["acting_batch1"] = bench_acting(d, dev)
    if secondary:
        out["secondary"] = secondary
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, B, S, H, budget_s=args.cpu_budget)
    print(json.dumps(out), flush=True)
    if world > 1:
        barrier()
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
