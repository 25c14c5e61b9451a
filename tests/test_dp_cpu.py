"""CPU (gloo, world_size 2) check of the data-parallel decomposition the
engine uses: each rank imagines its slice of the batch, the
lambda returns are all-gathered for the global update_S quantile, and the
actor/critic gradients -- scaled by 1/(B_global*H) -- are SUM-all-reduced.
The result must equal the single-process train_step on the whole batch."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import fixture_params, load_fixture
from oracle import dreamer_oracle as O


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _grads(P, z, h, r, c, a, mu, sg, Rg, scale):
    """Per-shard loss pieces with the global S normaliser; returns grads."""
    ap = [P["agent." + k] for k in O.ACTOR_KEYS]
    cp = [P["agent." + k] for k in O.CRITIC_KEYS]
    V_t = O.critic_value(h, z, P, "target_critic")
    R = O.lambda_returns(V_t, r, c)
    base = O.critic_value(h.detach(), z.detach(), P, "critic")[:, :-1]
    adv = (R - base).detach().squeeze(-1)
    logp = O.tanh_normal_logprob(a, mu, sg)
    S = O.update_S(1.0, Rg)
    norm = torch.max(torch.as_tensor(S), torch.tensor(1.0))
    la = torch.sum(-(logp * (adv / norm)) - (3e-4 * (-logp))) * scale
    lg = O.critic_logits(h.detach(), z.detach(), P, "critic")[:, :-1]
    th = O.twohot(O.symlog(R.detach()), P["agent.critic.buckets_crit"])
    lc = torch.sum(-torch.sum(th * torch.log_softmax(lg, -1), -1)) * scale
    ga = torch.autograd.grad(la, ap, allow_unused=True)
    gc = torch.autograd.grad(lc, cp, allow_unused=True)
    fix = lambda gs, ps: [torch.zeros_like(p) if g is None else g for g, p in zip(gs, ps)]
    return fix(ga, ap), fix(gc, cp), la.detach(), lc.detach(), R.detach()


def _setup():
    fx = load_fixture("small_epoch")
    P = fixture_params("small", fx)
    P = {k: (v.clone().requires_grad_(True) if k.startswith("agent.") and "buckets" not in k and "target" not in k
             else v) for k, v in P.items()}
    R_, C = int(fx["cfg_rows"]), int(fx["cfg_cols"])
    H = int(fx["cfg_H"])
    z0, h0 = torch.from_numpy(fx["z0"].copy()), torch.from_numpy(fx["h0"].copy())
    eps, q = torch.from_numpy(fx["eps"].copy()), torch.from_numpy(fx["q"].copy())
    return fx, P, R_, C, H, z0, h0, eps, q


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fx, P, R_, C, H, z0, h0, eps, q = _setup()
    B = z0.shape[0]
    b = B // world
    sl = slice(rank * b, (rank + 1) * b)
    C_ = q.shape[-1]
    qs = q.view(H, B, -1, C_)[:, sl].reshape(H, -1, C_)
    z, h, a, r, c, mu, sg = O.dream(z0[sl], h0[sl], P, eps[:, sl], qs, H, R_, C)
    V_t = O.critic_value(h, z, P, "target_critic")
    R_loc = O.lambda_returns(V_t, r, c).detach().contiguous()
    parts = [torch.empty_like(R_loc) for _ in range(world)]
    dist.all_gather(parts, R_loc)
    Rg = torch.cat(parts, 0)
    ga, gc, la, lc, _ = _grads(P, z, h, r, c, a, mu, sg, Rg, 1.0 / (B * H))
    flat = torch.cat([g.reshape(-1) for g in ga + gc] + [la.view(1), lc.view(1)])
    dist.all_reduce(flat)
    if rank == 0:
        torch.save(flat, out)
    dist.destroy_process_group()


def test_dp_decomposition_gloo(tmp_path):
    out = str(tmp_path / "flat.pt")
    mp.spawn(_worker, args=(2, _port(), out), nprocs=2, join=True)
    flat = torch.load(out)
    fx, P, R_, C, H, z0, h0, eps, q = _setup()
    B = z0.shape[0]
    z, h, a, r, c, mu, sg = O.dream(z0, h0, P, eps, q, H, R_, C)
    ts = O.train_step(z, h, r, c, a, mu, sg, P, 1.0, [P["agent." + k] for k in O.ACTOR_KEYS],
                      [P["agent." + k] for k in O.CRITIC_KEYS])
    ref = torch.cat([g.reshape(-1) for g in ts["grad_actor"] + ts["grad_critic"]]
                    + [ts["loss_actor"].view(1), ts["loss_critic"].view(1)])
    # shards differ from the whole batch only by fp32 summation order (MKL GEMM
    # blocking depends on the row count): ~1 ulp in the forward, 1e-6 in grads
    tol = 1e-5 * float(ref.abs().max())
    assert torch.allclose(flat, ref, rtol=1e-4, atol=tol), float((flat - ref).abs().max())
