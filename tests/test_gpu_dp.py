"""Data-parallel train_Agent on the real HIP path: 2 ranks (gloo, both on
cuda:0 of the one-GPU box) vs one process on the concatenated batch.
Philox noise is keyed by the global row, so both runs draw identical noise;
the all-gathered returns give the same global quantile, and the all-reduced
flat gradient differs from the single-device sum only in summation order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import dp_worker

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("pipelined", [False, True])
def test_two_rank_matches_single(pipelined, gpu, tmp_path):
    from dreamer_amd.engine import ImaginationEngine
    B = 8
    rng = np.random.RandomState(11)
    starts = [rng.randint(0, 64 - 8 + 1, size=B) for _ in range(3)]
    out = str(tmp_path / "dp.pt")
    mp.spawn(dp_worker.worker, args=(2, _port(), B, starts, out, "gloo", pipelined), nprocs=2, join=True)
    dp = torch.load(out, weights_only=False)
    d = dp_worker.make_dreamer(gpu, B)
    eng = ImaginationEngine(d, B=B)
    single = dp_worker.run_epochs(d, eng, starts)
    for (la1, lc1), (la2, lc2) in zip(single[0], dp[0]):
        assert abs(la1 - la2) <= 1e-4 * max(1.0, abs(la1)), (la1, la2)
        assert abs(lc1 - lc2) <= 1e-4 * max(1.0, abs(lc1)), (lc1, lc2)
    for a, b, name in zip(single[1:4], dp[1:4], ("actor", "critic", "target")):
        assert torch.allclose(a, b, rtol=0, atol=5e-6), (name, float((a - b).abs().max()))
    assert abs(single[4] - dp[4]) < 1e-6


def test_two_rank_world_model_matches_single(gpu, tmp_path):
    """WorldModel.training_step sharded over 2 ranks (mask and loss sums
    all-reduced between the phases, gradient all-reduced before the clip) vs
    one process on the whole batch: same losses, same parameters after 3 steps
    up to summation order."""
    B = 8
    rng = np.random.RandomState(12)
    starts = [rng.randint(0, 64 - 8 + 1, size=B) for _ in range(3)]
    out = str(tmp_path / "dpwm.pt")
    mp.spawn(dp_worker.wm_worker, args=(2, _port(), B, starts, out, "gloo"), nprocs=2, join=True)
    dp = torch.load(out, weights_only=True)
    d = dp_worker.make_dreamer(gpu, B)
    single = dp_worker.run_wm_steps(d, starts)
    for l1, l2 in zip(single[0], dp[0]):
        assert abs(l1 - l2) <= 1e-4 * max(1.0, abs(l1)), (l1, l2)
    err = float((single[1] - dp[1]).abs().max())
    assert err <= 5e-6, err


def test_two_rank_full_width_matches_single(gpu, tmp_path):
    """CarRacing widths at BASELINE configs[1]'s per-rank shape: 2 ranks x 32
    rows (S=64, H=15) vs one process on the 64-row batch, 2 epochs."""
    from dreamer_amd.engine import ImaginationEngine
    B = 64
    rng = np.random.RandomState(13)
    starts = [rng.randint(0, 1024 - 64 + 1, size=B) for _ in range(2)]
    out = str(tmp_path / "dpfull.pt")
    mp.spawn(dp_worker.worker, args=(2, _port(), B, starts, out, "gloo", False, True), nprocs=2, join=True)
    dp = torch.load(out, weights_only=False)
    d = dp_worker.make_dreamer(gpu, B, full=True)
    eng = ImaginationEngine(d, B=B)
    single = dp_worker.run_epochs(d, eng, starts)
    for (la1, lc1), (la2, lc2) in zip(single[0], dp[0]):
        assert abs(la1 - la2) <= 1e-4 * max(1e-3, abs(la1)), (la1, la2)
        assert abs(lc1 - lc2) <= 1e-4 * abs(lc1), (lc1, lc2)
    for a, b, name in zip(single[1:4], dp[1:4], ("actor", "critic", "target")):
        err = (a - b).abs()
        # Adam's first steps move a weight by ~lr whatever the gradient's size,
        # so a summation-order difference on a near-zero gradient can flip one
        # step's sign: bounded count, everything else at 1e-6
        bad = err > 1e-6 + 1e-6 * a.abs()
        assert int(bad.sum()) <= max(4, a.numel() // 20000), (name, int(bad.sum()), float(err.max()))
        assert float(err.max()) <= 4 * 1e-4 + 1e-6, (name, float(err.max()))
    assert abs(single[4] - dp[4]) < 1e-5 * abs(single[4])


def test_eight_rank_configs2_matches_single(gpu, tmp_path):
    """BASELINE configs[2] at its real decomposition: global B = 512 (S = 64,
    H = 15, CarRacing widths, 64 x 64 frames) as 8 ranks x 64 rows -- one
    process per rank, all on the box's one GPU, gloo standing in for RCCL --
    against ONE process running the whole 512-row batch, for 2 train_Agent
    epochs (Dreamer.py:264-287).  The exchange under test is the engine's:
    all-gather of the lambda returns for the global quantile of update_S
    (Agent.py:83-84) and one all-reduce of the flat [actor | critic | loss]
    gradient before clip_grad_norm_ (Agent.py:141-148).  Philox noise is keyed
    by the global row, so both runs draw the same variates.

    Epoch 1 (identical parameters): losses within 1e-4 relative, S within
    1e-6 relative, clipped gradients |d| <= 1e-4 |ref| + 1e-5 max|ref| per
    buffer.  Epoch 2 starts from parameters that may differ by an Adam sign
    flip on near-zero gradients (below), so its losses get 2e-3 relative and
    its S 1e-5.  Final actor / critic / target parameters: |d| <= 1e-6 +
    1e-6 |p| except a bounded count of sign-flipped elements, each <= 4 lr."""
    from dreamer_amd.engine import ImaginationEngine
    B, world = 512, 8
    rng = np.random.RandomState(14)
    starts = [rng.randint(0, 1024 - 64 + 1, size=B) for _ in range(2)]
    out = str(tmp_path / "dp8.pt")
    mp.spawn(dp_worker.worker, args=(world, _port(), B, starts, out, "gloo", False, True), nprocs=world, join=True)
    dp = torch.load(out, weights_only=True)
    d = dp_worker.make_dreamer(gpu, B, full=True)
    eng = ImaginationEngine(d, B=B)
    single = dp_worker.run_epochs(d, eng, starts)
    (la1, lc1), (la2, lc2) = single[0][0], dp[0][0]
    assert abs(la1 - la2) <= 1e-4 * max(1e-3, abs(la1)), ("epoch 1 actor loss", la1, la2)
    assert abs(lc1 - lc2) <= 1e-4 * abs(lc1), ("epoch 1 critic loss", lc1, lc2)
    assert abs(single[6][0] - dp[6][0]) <= 1e-6 * abs(single[6][0]), ("epoch 1 S", single[6][0], dp[6][0])
    g1, g2 = single[5][0], dp[5][0]
    na = d.agent.fa.numel
    for lo, hi, name in ((0, na, "actor"), (na, g1.numel(), "critic")):
        a, b = g1[lo:hi], g2[lo:hi]
        tol = 1e-4 * a.abs() + 1e-5 * float(a.abs().max())
        bad = (a - b).abs() > tol
        assert not bool(bad.any()), (f"epoch 1 clipped {name} grads", int(bad.sum()), float((a - b).abs().max()))
    (la1, lc1), (la2, lc2) = single[0][1], dp[0][1]
    assert abs(la1 - la2) <= 2e-3 * max(1e-3, abs(la1)), ("epoch 2 actor loss", la1, la2)
    assert abs(lc1 - lc2) <= 2e-3 * abs(lc1), ("epoch 2 critic loss", lc1, lc2)
    assert abs(single[4] - dp[4]) <= 1e-5 * abs(single[4]), ("epoch 2 S", single[4], dp[4])
    flips = {}
    for a, b, name in zip(single[1:4], dp[1:4], ("actor", "critic", "target")):
        err = (a - b).abs()
        bad = err > 1e-6 + 1e-6 * a.abs()
        flips[name] = int(bad.sum())
        assert flips[name] <= max(8, a.numel() // 10000), (name, flips[name], float(err.max()))
        assert float(err.max()) <= 4 * 1e-4 + 1e-6, (name, float(err.max()))
    print(f"configs[2] 8x64 vs 1x512: losses e1 {single[0][0]} / {dp[0][0]}, e2 {single[0][1]} / {dp[0][1]}, "
          f"S {single[4]:.6f} / {dp[4]:.6f}, sign-flipped params {flips}")
