"""Timing probe (GPU box): can the world-model-only work of epoch e+1 (conv
encoder, posterior scan) run beside the actor-critic chain of epoch e
(imagine .. optim) on separate (optionally CU-masked, prioritised) streams?

Timing only: the concurrent replays share buffers, so the numbers are not
results.   python tools/overlap_probe.py
"""
import ctypes as C
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

hip = C.CDLL("libamdhip64.so")


def masked_stream(bits, prio=0):
    words = (C.c_uint32 * 8)()
    for b in bits:
        words[b // 32] |= (1 << (b % 32))
    s = C.c_void_p()
    err = hip.hipExtStreamCreateWithCUMask(C.byref(s), 8, words)
    assert err == 0, err
    if prio:
        # re-create with priority is not possible with a mask; report it
        pass
    return torch.cuda.ExternalStream(s.value)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from dreamer_amd import Dreamer
    from dreamer_amd.engine import ImaginationEngine
    cfg = dict(bench.CAR_RACER)
    B = int(os.environ.get("B", "64"))
    cfg.update(batch_size=B)
    torch.manual_seed(0)
    d = Dreamer(cfg, dev)
    fr, ac, rw, ct = bench.synthetic_replay(4096, cfg["observation_dims"], 3)
    d.buffer.load_arrays(fr, ac, rw, ct)
    d.buffer._mirror()
    eng = ImaginationEngine(d, B=B)
    for _ in range(3):
        eng.run(d.buffer.sample_start_indices(B))
    torch.cuda.synchronize()
    chain = eng.graph[1:]
    cap = torch.cuda.Stream(dev)
    cap.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cap):
        genc, gscan = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(genc, stream=cap):
            eng._encode_chunk(0, eng.T, cap.cuda_stream)
        with torch.cuda.graph(gscan, stream=cap):
            eng._scan_chunk(0, eng.T, cap.cuda_stream)
    torch.cuda.synchronize()
    N = 20

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / N * 1e3, 3)

    def run_chain():
        for c in chain:
            c.replay()

    out = {"B": B}
    out["seq"] = timed(lambda: [(genc.replay(), gscan.replay(), run_chain()) for _ in range(N)])
    out["enc"] = timed(lambda: [genc.replay() for _ in range(N)])
    out["scan"] = timed(lambda: [gscan.replay() for _ in range(N)])
    out["chain"] = timed(lambda: [run_chain() for _ in range(N)])

    def two(s1, s2, first, second):
        def f():
            for _ in range(N):
                with torch.cuda.stream(s1):
                    first()
                with torch.cuda.stream(s2):
                    second()
        return f

    def three(s1, s2, s3):
        def f():
            for _ in range(N):
                with torch.cuda.stream(s1):
                    genc.replay()
                with torch.cuda.stream(s2):
                    gscan.replay()
                with torch.cuda.stream(s3):
                    run_chain()
        return f

    for nch in [int(x) for x in os.environ.get("CHUNKS", "2,4,8").split(",")]:
        ge = torch.cuda.CUDAGraph()
        with torch.cuda.stream(cap):
            with torch.cuda.graph(ge, stream=cap):
                for t0, t1 in eng.warm_chunks(eng.T, (eng.T + nch - 1) // nch):
                    eng._encode_chunk(t0, t1, cap.cuda_stream)
        torch.cuda.synchronize()
        warm = lambda: (ge.replay(), gscan.replay())
        out[f"chunks{nch} enc"] = timed(lambda: [ge.replay() for _ in range(N)])
        out[f"chunks{nch} warm|chain"] = timed(two(torch.cuda.Stream(dev), torch.cuda.Stream(dev), warm, run_chain))
        out[f"chunks{nch} warm|chain(hi)"] = timed(two(torch.cuda.Stream(dev), torch.cuda.Stream(dev, priority=-1),
                                                       warm, run_chain))
        print(json.dumps(out), flush=True)
    # the scan alone beside the chain, and the encoder alone beside the chain
    out["scan|chain"] = timed(two(torch.cuda.Stream(dev), torch.cuda.Stream(dev), gscan.replay, run_chain))
    out["enc|chain"] = timed(two(torch.cuda.Stream(dev), torch.cuda.Stream(dev), genc.replay, run_chain))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
