"""Probe: does the per-step chain run faster as several batch lanes on
separate streams?  Times the imagination unroll (dr_imagine_fwd), the
posterior scan (dr_observe_scan) and the BPTT (dr_imagine_bwd) at B = 256 as
one chain against 2 x 128 and 4 x 64 row lanes, each lane its own buffers
and workspace, replayed (a) as one graph per lane on its own stream, (b) as
ONE graph whose lanes fork / join on events inside the capture.

  python tools/lanes_probe.py [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from dreamer_amd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, S, H = args.B, 64, 15
    cfg, d = bench.make_dreamer(bench.CAR_RACER, dev, B, S, H, 64, 1, 1, 0, None, "fp32")
    for _ in range(3):
        d.train_Agent()
    torch.cuda.synchronize()
    eng = d._engine
    dd = eng.d
    wm = d.world_model.packed()
    ac = d.agent.actor_struct()
    acg = d.agent.actor_struct(grad=True)
    Ld, Hd, A, T = dd.rows * dd.cols, dd.hidden, dd.action, S // 2
    f = lambda *s: torch.zeros(*s, device=dev)

    def lane(b0, Bl):
        x = dict(b0=b0, B=Bl)
        x["lat"], x["hid"] = f(Bl, H + 1, Ld), f(Bl, H + 1, Hd)
        for k in ("act", "mu", "sig", "gmu", "gsig"):
            x[k] = f(Bl, H, A)
        x["rew"], x["cont"] = f(Bl, H), f(Bl, H)
        x["tape"] = torch.zeros(L.query("dr_imagine_tape_bytes", dd, Bl, H), dtype=torch.uint8, device=dev)
        x["ws"] = torch.zeros(L.query("dr_imagine_workspace_bytes", dd, Bl, H), dtype=torch.uint8, device=dev)
        x["wso"] = torch.zeros(L.query("dr_observe_workspace_bytes", dd, Bl), dtype=torch.uint8, device=dev)
        x["feat"] = torch.randn(T, Bl, dd.enc_hidden, device=dev)
        x["z0"], x["h0"] = f(Bl, Ld), f(Bl, Hd)
        x["gmu"].normal_(0, 1e-3)
        x["gsig"].normal_(0, 1e-3)
        return x

    def imagine(x, st):
        b0 = x["b0"]
        nz = L.dr_noise(None, None, eng.rng.state.data_ptr(), b0, 2 << 24)
        L.call("dr_imagine_fwd", dd, wm, ac, x["B"], H, L.ptr(eng.z0) + b0 * Ld * 4, L.ptr(eng.h0) + b0 * Hd * 4,
               nz, 0, L.ptr(x["lat"]), L.ptr(x["hid"]), L.ptr(x["act"]), L.ptr(x["rew"]), L.ptr(x["cont"]),
               L.ptr(x["mu"]), L.ptr(x["sig"]), L.ptr(x["tape"]), L.ptr(x["ws"]), x["ws"].numel(), st)

    def scan(x, st):
        b0 = x["b0"]
        nz = L.dr_noise(None, None, eng.rng.state.data_ptr(), b0, 1 << 24)
        L.call("dr_observe_scan", dd, wm, x["B"], T, L.ptr(x["feat"]), L.ptr(eng.act_win) + b0 * S * A * 4, S * A, A,
               None, None, nz, L.ptr(x["z0"]), L.ptr(x["h0"]), None, L.ptr(x["wso"]), x["wso"].numel(), st)

    def bptt(x, st):
        L.call("dr_imagine_bwd", dd, wm, ac, x["B"], H, L.ptr(x["lat"]), L.ptr(x["hid"]), L.ptr(x["act"]),
               L.ptr(x["gmu"]), L.ptr(x["gsig"]), None, None, None, L.ptr(x["tape"]), acg, L.ptr(x["ws"]),
               x["ws"].numel(), st)

    res = {}
    for nl in (1, 2, 4):
        Bl = B // nl
        lanes = [lane(i * Bl, Bl) for i in range(nl)]
        streams = [torch.cuda.Stream(dev) for _ in range(nl)]
        # eager once (populates the imagination outputs the BPTT reads)
        for x, s in zip(lanes, streams):
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                imagine(x, s.cuda_stream)
        torch.cuda.synchronize()
        for name, fn in (("imagine", imagine), ("scan", scan), ("bptt", bptt)):
            # (a) one graph per lane on its own stream
            graphs = []
            for x, s in zip(lanes, streams):
                g = torch.cuda.CUDAGraph()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.graph(g, stream=s):
                    fn(x, s.cuda_stream)
                graphs.append(g)
            torch.cuda.synchronize()
            main = torch.cuda.current_stream()

            def run_a():
                ev = torch.cuda.Event()
                ev.record(main)
                for g, s in zip(graphs, streams):
                    s.wait_event(ev)
                    with torch.cuda.stream(s):
                        g.replay()
                for s in streams:
                    main.wait_stream(s)

            # (b) one graph, lanes forked on events inside the capture
            gb = torch.cuda.CUDAGraph()
            cap = streams[0]
            cap.wait_stream(main)
            with torch.cuda.graph(gb, stream=cap):
                ev0 = torch.cuda.Event()
                ev0.record(cap)
                for x, s in zip(lanes[1:], streams[1:]):
                    s.wait_event(ev0)
                    with torch.cuda.stream(s):
                        fn(x, s.cuda_stream)
                fn(lanes[0], cap.cuda_stream)
                for s in streams[1:]:
                    e = torch.cuda.Event()
                    e.record(s)
                    cap.wait_event(e)
            torch.cuda.synchronize()

            def run_b():
                gb.replay()

            for tag, run in (("per_lane_graphs", run_a), ("forked_graph", run_b)):
                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record(main)
                for _ in range(args.reps):
                    run()
                t1.record(main)
                torch.cuda.synchronize()
                ms = t0.elapsed_time(t1) / args.reps
                res[f"{name}_lanes{nl}_{tag}"] = round(ms, 4)
                print(f"{name:8s} lanes={nl} {tag:16s} {ms:8.4f} ms", flush=True)
            assert torch.isfinite(lanes[0]["hid"]).all()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
