"""The data-parallel collective path over RCCL (torch.distributed backend
"nccl") on the one-GPU box: a world_size-1 process group with the
collectives forced on.  Run on the MI355X box: pytest -m gpu.

Until round 4 the nccl branch of bench.py and the engine / world-model
collectives had only ever run under gloo (tests/test_gpu_dp.py).  Here the
same code runs over RCCL, between captured phase graphs:

* train_Agent epochs (ImaginationEngine.run, graph replay): the all-gather of
  the lambda returns (global quantile of update_S, Agent.py:83-84) and the
  all-reduce of the flat [actor | critic | losses] gradient buffer before
  clip_grad_norm_;
* the world-model step (WorldModel.train_step_ring): the all-reduced mask sum
  (WorldModel.py:185) and loss sums between the forward phases, and the three
  gradient buckets all-reduced asynchronously (async_op=True, RCCL's stream)
  while the next backward stage computes, each wait()ed before clip.

With one rank every collective is an identity, so the results must equal the
plain single-GPU run bit for bit (same weights, windows and Philox state)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_group(gpu):
    import torch.distributed as dist
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29641", rank=0, world_size=1, device_id=gpu)
    assert dist.get_backend() == "nccl"
    yield dist.group.WORLD
    dist.destroy_process_group()


def _pair(gpu, B, group):
    import bench
    from dreamer_amd.engine import ImaginationEngine
    _, plain = bench.make_dreamer(bench.CAR_RACER, gpu, B, 64, 15, 64, 1, 1, 0, None, "fp32")
    _, dp = bench.make_dreamer(bench.CAR_RACER, gpu, B, 64, 15, 64, 1, 1, 0, None, "fp32")
    dp.world = (0, 1, group)
    dp.world_model.set_data_parallel(0, 1, group, force=True)
    dp._engine = ImaginationEngine(dp, B=B, world=(0, 1, group))
    assert dp._engine.dp and not plain._engine.dp
    return plain, dp


def _state_equal(a, b, what):
    sa, sb = a.state_dict(), b.state_dict()
    bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
    assert not bad, f"{what}: {len(bad)} tensors differ, e.g. {bad[:4]}"


def test_rccl_train_agent_epochs_match_single(gpu, rccl_group):
    """Three graph-replayed train_Agent epochs with the RCCL collectives
    between the phase graphs == the same epochs without them, bitwise."""
    from dreamer_amd import hip
    B = 256
    plain, dp = _pair(gpu, B, rccl_group)
    rng = np.random.RandomState(7)
    starts = [rng.randint(0, 4096 - 64, size=B) for _ in range(3)]
    out = {}
    for name, d in (("plain", plain), ("rccl", dp)):
        hip.rng(gpu).reseed(0xC0FFEE)
        losses = []
        for st in starts:
            la, lc = d._engine.run(st)
            losses.append((la.clone(), lc.clone()))
        torch.cuda.synchronize()
        out[name] = (losses, float(d.agent.S_dev))
    for (a1, c1), (a2, c2) in zip(out["plain"][0], out["rccl"][0]):
        assert torch.equal(a1, a2) and torch.equal(c1, c2), (a1, a2, c1, c2)
    assert out["plain"][1] == out["rccl"][1]
    _state_equal(plain, dp, "agent after 3 epochs")
    print(f"RCCL world 1: 3 epochs bitwise equal, losses {[float(x[0]) for x in out['rccl'][0]]}, S {out['rccl'][1]}")


def test_rccl_world_model_step_matches_single(gpu, rccl_group):
    """Two WorldModel.train_step_ring steps with the RCCL stats all-reduces and
    the three async gradient buckets == the plain step, bitwise."""
    from dreamer_amd import hip
    B = 64
    plain, dp = _pair(gpu, B, rccl_group)
    rng = np.random.RandomState(9)
    starts = [rng.randint(0, 4096 - 64, size=B) for _ in range(2)]
    res = {}
    for name, d in (("plain", plain), ("rccl", dp)):
        hip.adhoc(gpu).reseed(0xBEEF)
        ls = [d.world_model.train_step_ring(d.buffer, st) for st in starts]
        torch.cuda.synchronize()
        res[name] = [float(x) for x in ls]
    assert res["plain"] == res["rccl"], res
    _state_equal(plain, dp, "world model after 2 steps")
    print(f"RCCL world 1: 2 WM steps bitwise equal, losses {res['rccl']}")
