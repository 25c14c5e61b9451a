"""dr_adamw / dr_ema pinned directly (the fused optimiser was only
checked after one step inside whole-epoch tests, at a 2*lr band).

The reference's optimisers are torch.optim.AdamW on CPU (Agent.py:63-76,
WorldModel.py:64-66) with clip_grad_norm_ before the step (Agent.py:147-148)
and an EMA target critic (Agent.py:153).  Here the C-ABI kernels run 4
consecutive steps on 40,000 parameters with fresh gradients each step
(so the device step counter's bias correction at steps 2..4 is exercised)
against torch.optim.AdamW itself and the oracle's restatement, with a large
weight decay so a missing / misplaced decay shows.  Tolerances: parameters
within 2 ulp-scale (4e-7 relative + 1e-9), and the per-step UPDATE within 1e-3
of its own size (plus the rounding of p) -- a wrong sign, bias correction or
decay is O(1) of it.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _adamw_gpu(p, g, m, v, step, hyper, lr, b1, b2, eps, wd, sqnorm=None, max_norm=100.0, skip=None):
    from dreamer_amd import _lib as L
    from dreamer_amd import hip
    L.call("dr_adamw", p.numel(), L.ptr(p), L.ptr(g), L.ptr(m), L.ptr(v), L.ptr(sqnorm), max_norm, lr, b1, b2, eps,
           wd, L.ptr(step), L.ptr(hyper), L.ptr(skip), hip.stream())


@pytest.mark.parametrize("clip", [False, True])
def test_adamw_multistep_matches_torch(gpu, clip):
    import oracle.dreamer_oracle as O
    n, lr, b1, b2, eps, wd, max_norm = 40_000, 1e-3, 0.9, 0.999, 1e-5, 0.05, 2.0
    gen = torch.Generator().manual_seed(11)
    p0 = torch.randn(n, generator=gen)
    ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([ref], lr=lr, betas=(b1, b2), eps=eps, weight_decay=wd, foreach=False)
    po, mo, vo = p0.clone(), torch.zeros(n), torch.zeros(n)
    p, m, v = p0.to(gpu), torch.zeros(n, device=gpu), torch.zeros(n, device=gpu)
    step = torch.zeros(1, dtype=torch.int32, device=gpu)
    hyper = torch.zeros(2, device=gpu)
    for k in range(1, 5):
        g = torch.randn(n, generator=gen) * (3.0 if clip else 0.01)
        if clip:  # clip_grad_norm_ (Agent.py:147-148): g * min(1, max_norm / (|g| + 1e-6))
            gc, _ = O.clip_grad_norm([g], max_norm)
            gc = gc[0]
        else:
            gc = g
        prev = ref.detach().clone()
        ref.grad = gc.clone()
        opt.step()
        po, mo, vo = O.adamw_step(po, gc, mo, vo, k, lr, (b1, b2), eps, wd)
        gd = g.to(gpu)
        sq = (gd.double() ** 2).sum().float().reshape(1) if clip else None
        pg_prev = p.clone()
        _adamw_gpu(p, gd, m, v, step, hyper, lr, b1, b2, eps, wd, sqnorm=sq, max_norm=max_norm)
        torch.cuda.synchronize()
        pc = p.cpu()
        assert int(step.item()) == k
        if clip:  # g scaled in place, like clip_grad_norm_ on p.grad
            np.testing.assert_allclose(gd.cpu().numpy(), gc.numpy(), rtol=2e-6, atol=1e-9)
        for name, want in (("torch.optim.AdamW", ref.detach()), ("oracle adamw_step", po)):
            err = (pc - want).abs()
            assert bool((err <= 4e-7 * want.abs() + 1e-9).all()), \
                f"step {k}: params vs {name}: max abs err {float(err.max()):.3g}"
        upd_ref = ref.detach() - prev
        upd = pc - pg_prev.cpu()
        # the update to within 1e-3 of itself, up to the rounding of p (ulp ~ 1.2e-7 |p|)
        bad = (upd - upd_ref).abs() > 1e-3 * upd_ref.abs() + 4e-7 * pc.abs()
        assert not bool(bad.any()), f"step {k}: {int(bad.sum())} updates off by more than 1e-3 of themselves"
        # lerp cancels near m = 0: absolute slack of a few ulp of g (|g| ~ 0.01 -> ulp 1e-9)
        np.testing.assert_allclose(m.cpu().numpy(), mo.numpy(), rtol=1e-6, atol=1e-8)
        np.testing.assert_allclose(v.cpu().numpy(), vo.numpy(), rtol=2e-6, atol=1e-14)
        # the update is not the decay alone: bias-corrected Adam moves every weight by about lr
        assert float(upd_ref.abs().median()) > 0.3 * lr


def test_adamw_skip_leaves_state(gpu):
    n = 4096
    p = torch.randn(n, device=gpu)
    p0 = p.clone()
    g = torch.randn(n, device=gpu)
    m, v = torch.zeros(n, device=gpu), torch.zeros(n, device=gpu)
    step = torch.zeros(1, dtype=torch.int32, device=gpu)
    hyper = torch.zeros(2, device=gpu)
    skip = torch.ones(1, dtype=torch.int32, device=gpu)
    _adamw_gpu(p, g, m, v, step, hyper, 1e-3, 0.9, 0.999, 1e-5, 1e-6, skip=skip)
    torch.cuda.synchronize()
    assert torch.equal(p, p0) and int(step.item()) == 0 and float(m.abs().sum()) == 0.0


def test_ema_matches_reference_formula(gpu):
    """target <- (1 - tau) * target + tau * src (Agent.py:153 soft_update_target), 3 rounds."""
    from dreamer_amd import _lib as L
    from dreamer_amd import hip
    gen = torch.Generator().manual_seed(3)
    t = torch.randn(10_000, generator=gen)
    tg = t.to(gpu)
    tau = 0.02
    for _ in range(3):
        s = torch.randn(10_000, generator=gen)
        t = t * (1 - tau) + tau * s
        L.call("dr_ema", tg.numel(), L.ptr(tg), L.ptr(s.to(gpu)), 1 - tau, tau, None, hip.stream())
    torch.cuda.synchronize()
    np.testing.assert_allclose(tg.cpu().numpy(), t.numpy(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("bad_loss", [False, True])
def test_ac_optimiser_step_equals_five_calls(gpu, bad_loss):
    """dr_ac_optimiser_step (the engine's optimiser tail: clip stats + both
    AdamW preludes, then both AdamW updates and the target EMA in one pass)
    is bitwise the sequence it replaces -- dr_clip_stats, dr_adamw(critic),
    dr_adamw(actor), dr_ema -- over 3 steps with fresh gradients (clipping
    active on one net), and a non-finite loss skips everything in both."""
    from dreamer_amd import _lib as L
    from dreamer_amd import hip
    na, nc = 50_000, 30_004
    hp = dict(lr_a=4e-5, lr_c=1e-4, b1=0.9, b2=0.999, eps=1e-5, wd=0.01)
    gen = torch.Generator().manual_seed(5)

    def state():
        t = {k: torch.randn(n, generator=gen).to(gpu) for k, n in (("pa", na), ("pc", nc), ("tgt", nc))}
        for k, n in (("ma", na), ("va", na), ("mc", nc), ("vc", nc)):
            t[k] = torch.zeros(n, device=gpu)
        t.update(sa=torch.zeros(1, dtype=torch.int32, device=gpu), sc=torch.zeros(1, dtype=torch.int32, device=gpu),
                 ha=torch.zeros(2, device=gpu), hc=torch.zeros(2, device=gpu), sq=torch.zeros(2, device=gpu),
                 skip=torch.zeros(1, dtype=torch.int32, device=gpu), scr=torch.zeros(1024, device=gpu))
        return t

    A, Bs = state(), None
    Bs = {k: v.clone() for k, v in A.items()}
    st = hip.stream()
    for it in range(3):
        ga = (torch.randn(na, generator=gen) * (30.0 if it == 1 else 0.01)).to(gpu)
        gc = (torch.randn(nc, generator=gen) * 0.02).to(gpu)
        loss = torch.tensor([0.5, float("nan") if (bad_loss and it == 2) else 1.5], device=gpu)
        gA, gcA, gB, gcB = ga.clone(), gc.clone(), ga.clone(), gc.clone()
        # the five calls
        L.call("dr_clip_stats", na, L.ptr(gA), nc, L.ptr(gcA), 2, L.ptr(loss), L.ptr(A["sq"]), L.ptr(A["skip"]),
               L.ptr(A["scr"]), st)
        L.call("dr_adamw", nc, L.ptr(A["pc"]), L.ptr(gcA), L.ptr(A["mc"]), L.ptr(A["vc"]), L.ptr(A["sq"]) + 4, 100.0,
               hp["lr_c"], hp["b1"], hp["b2"], hp["eps"], hp["wd"], L.ptr(A["sc"]), L.ptr(A["hc"]), L.ptr(A["skip"]),
               st)
        L.call("dr_adamw", na, L.ptr(A["pa"]), L.ptr(gA), L.ptr(A["ma"]), L.ptr(A["va"]), L.ptr(A["sq"]), 100.0,
               hp["lr_a"], hp["b1"], hp["b2"], hp["eps"], hp["wd"], L.ptr(A["sa"]), L.ptr(A["ha"]), L.ptr(A["skip"]),
               st)
        L.call("dr_ema", nc, L.ptr(A["tgt"]), L.ptr(A["pc"]), float(1.0 - 0.02), 0.02, L.ptr(A["skip"]), st)
        # the fused step
        L.call("dr_ac_optimiser_step", na, L.ptr(Bs["pa"]), L.ptr(gB), L.ptr(Bs["ma"]), L.ptr(Bs["va"]),
               L.ptr(Bs["sa"]), L.ptr(Bs["ha"]), hp["lr_a"], hp["b1"], hp["b2"], hp["eps"], hp["wd"],
               nc, L.ptr(Bs["pc"]), L.ptr(gcB), L.ptr(Bs["mc"]), L.ptr(Bs["vc"]), L.ptr(Bs["sc"]), L.ptr(Bs["hc"]),
               hp["lr_c"], hp["b1"], hp["b2"], hp["eps"], hp["wd"], 100.0, L.ptr(Bs["tgt"]), float(1.0 - 0.02),
               0.02, 2, L.ptr(loss), L.ptr(Bs["sq"]), L.ptr(Bs["skip"]), L.ptr(Bs["scr"]), st)
        torch.cuda.synchronize()
        assert torch.equal(gA, gB) and torch.equal(gcA, gcB), f"step {it}: clipped gradients differ"
        for k in A:
            if k == "scr":
                continue
            assert torch.equal(A[k], Bs[k]), f"step {it}: {k} differs"
    assert int(A["sa"].item()) == (2 if bad_loss else 3)
