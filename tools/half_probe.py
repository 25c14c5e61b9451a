"""Does the B = 256 chain gain from running as two independent B / 2 chains on
two streams?  The posterior scan, the imagination unroll and the BPTT reverse
loop are per-row (Dreamer.py:158-164, 255-261; Agent.py:96-154 backward), and
at B = 256 their launches are latency-bound, so two half-batch chains could
overlap.  Times (HIP events, graph replays, launch form):

  full    one B-row call
  seq     the two halves one after the other on one stream
  conc    the two halves on two streams at once

for the warm start's scan, the unroll and the BPTT (+ actor weight gradients).
python tools/half_probe.py [B] [fp32|bf16]   (GPU box)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dreamer_amd import _lib as L  # noqa: E402
from dreamer_amd import hip  # noqa: E402
from dreamer_amd.engine import DREAM_STREAM, WARM_STREAM  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    np.random.seed(1)
    _, d = bench.make_dreamer(bench.CAR_RACER, dev, B, 64, 15, 64, 1, 1, 0, None, prec)
    eng = d._engine
    for _ in range(3):
        eng.run(d.buffer.sample_start_indices(B))
    torch.cuda.synchronize()
    dm = L.dr_dims.from_buffer_copy(eng.d)
    dm.launch_form = 1
    wm, ag = d.world_model.packed(), d.agent
    H, T, S, A = eng.H, eng.T, eng.S, dm.action
    Lat, Hd = dm.rows * dm.cols, dm.hidden
    Bh = B // 2
    f32 = lambda *s: torch.zeros(*s, device=dev)
    # per-half buffers (rows r0 .. r0 + Bh of the engine's tensors)
    halves = []
    for r0 in (0, Bh):
        h = dict(r0=r0)
        h["feat"] = f32(T * Bh, dm.enc_hidden)
        h["ws_enc"] = torch.zeros(L.query("dr_encoder_workspace_bytes", dm, T * Bh), dtype=torch.uint8, device=dev)
        h["ws_obs"] = torch.zeros(L.query("dr_observe_workspace_bytes", dm, Bh), dtype=torch.uint8, device=dev)
        h["z0"], h["h0"] = f32(Bh, Lat), f32(Bh, Hd)
        h["tape"] = torch.zeros(L.query("dr_imagine_tape_bytes", dm, Bh, H), dtype=torch.uint8, device=dev)
        h["ws_im"] = torch.zeros(L.query("dr_imagine_workspace_bytes", dm, Bh, H), dtype=torch.uint8, device=dev)
        h["grad"] = torch.zeros_like(ag.fa.flat)
        halves.append(h)
    f = ag.fa

    def grad_struct(buf):
        gp = lambda n: buf.data_ptr() + 4 * f.offsets[n]
        return L.dr_actor(*(L.dr_linear(gp(w), gp(b)) for w, b in (
            ("base_net.0.weight", "base_net.0.bias"), ("base_net.1.weight", "base_net.1.bias"),
            ("base_net.3.weight", "base_net.3.bias"), ("base_net.4.weight", "base_net.4.bias"),
            ("mu_head.weight", "mu_head.bias"), ("log_sig_head.weight", "log_sig_head.bias"))))

    off = lambda t, r0, per: t.data_ptr() + 4 * r0 * per

    def enc_half(h, st):
        fr = d.buffer.frames_struct(eng.starts)
        fr.starts = eng.starts.data_ptr() + 8 * h["r0"]
        L.call("dr_encoder_features", dm, wm, fr, Bh, T, L.ptr(h["feat"]), L.ptr(h["ws_enc"]), h["ws_enc"].numel(), st)

    def scan_half(h, st):
        nz = L.dr_noise(None, None, eng.rng.state.data_ptr(), h["r0"], WARM_STREAM)
        L.call("dr_observe_scan", dm, wm, Bh, T, L.ptr(h["feat"]), off(eng.act_win, h["r0"], S * A), S * A, A, None,
               None, nz, L.ptr(h["z0"]), L.ptr(h["h0"]), None, L.ptr(h["ws_obs"]), h["ws_obs"].numel(), st)

    def imagine_half(h, st):
        r0 = h["r0"]
        nz = L.dr_noise(None, None, eng.rng.state.data_ptr(), r0, DREAM_STREAM)
        L.call("dr_imagine_fwd", dm, wm, ag.actor_struct(), Bh, H, off(eng.z0, r0, Lat), off(eng.h0, r0, Hd), nz, 0,
               off(eng.latents, r0, (H + 1) * Lat), off(eng.hiddens, r0, (H + 1) * Hd), off(eng.actions, r0, H * A),
               off(eng.rewards, r0, H), off(eng.continues, r0, H), off(eng.mus, r0, H * A),
               off(eng.sigmas, r0, H * A), L.ptr(h["tape"]), L.ptr(h["ws_im"]), h["ws_im"].numel(), st)

    def bptt_half(h, st):
        r0 = h["r0"]
        L.call("dr_imagine_bwd", dm, wm, ag.actor_struct(), Bh, H, off(eng.latents, r0, (H + 1) * Lat),
               off(eng.hiddens, r0, (H + 1) * Hd), off(eng.actions, r0, H * A), off(eng.g_mu, r0, H * A),
               off(eng.g_sig, r0, H * A), None, None, None, L.ptr(h["tape"]), grad_struct(h["grad"]),
               L.ptr(h["ws_im"]), h["ws_im"].numel(), st)

    full_tape = eng.tape

    def scan_full(st):
        nz = L.dr_noise(None, None, eng.rng.state.data_ptr(), 0, WARM_STREAM)
        L.call("dr_observe_scan", dm, wm, B, T, L.ptr(eng.feat), L.ptr(eng.act_win), S * A, A, None, None, nz,
               L.ptr(eng.z0), L.ptr(eng.h0), None, L.ptr(eng.ws_obs), eng.ws_obs.numel(), st)

    def imagine_full(st):
        eng.imagine(d=dm)

    def bptt_full(st):
        L.call("dr_imagine_bwd", dm, wm, ag.actor_struct(), B, H, L.ptr(eng.latents), L.ptr(eng.hiddens),
               L.ptr(eng.actions), L.ptr(eng.g_mu), L.ptr(eng.g_sig), None, None, None, L.ptr(full_tape),
               ag.actor_struct(grad=True), L.ptr(eng.ws_im), eng.ws_im.numel(), st)

    # warm the half encoders / tapes once eagerly
    for h in halves:
        enc_half(h, hip.stream())
        scan_half(h, hip.stream())
        imagine_half(h, hip.stream())
        bptt_half(h, hip.stream())
    torch.cuda.synchronize()

    def capture(fn):
        cs = torch.cuda.Stream(dev)
        cs.wait_stream(torch.cuda.current_stream(dev))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(cs):
            with torch.cuda.graph(g, stream=cs):
                fn(cs.cuda_stream)
        torch.cuda.current_stream(dev).wait_stream(cs)
        return g

    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    main = torch.cuda.current_stream(dev)

    def timed(run, reps=20):
        run()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main)
        for _ in range(reps):
            run()
        b.record(main)
        b.synchronize()
        return a.elapsed_time(b) / reps

    res = {}
    for name, full_fn, half_fn in (("scan", scan_full, scan_half), ("imagine", imagine_full, imagine_half),
                                   ("bptt", bptt_full, bptt_half)):
        gf = capture(full_fn)
        gh = [capture(lambda st, h=h: half_fn(h, st)) for h in halves]

        def run_seq():
            gh[0].replay()
            gh[1].replay()

        def run_conc():
            s1.wait_stream(main)
            s2.wait_stream(main)
            with torch.cuda.stream(s1):
                gh[0].replay()
            with torch.cuda.stream(s2):
                gh[1].replay()
            main.wait_stream(s1)
            main.wait_stream(s2)

        res[name] = (timed(gf.replay), timed(run_seq), timed(run_conc))
        print(f"{prec} B={B} {name:8s} full {res[name][0]:7.3f} ms | halves seq {res[name][1]:7.3f} | "
              f"halves concurrent {res[name][2]:7.3f}", flush=True)
    # the encoder as two half calls (the halves' scans need contiguous [T][B/2] features)
    ge = capture(lambda st: L.call("dr_encoder_features", dm, wm, d.buffer.frames_struct(eng.starts), B, T,
                                   L.ptr(eng.feat), L.ptr(eng.ws_enc), eng.ws_enc.numel(), st))
    geh = capture(lambda st: [enc_half(h, st) for h in halves])
    print(f"{prec} B={B} encoder  full {timed(ge.replay):7.3f} ms | two half calls {timed(geh.replay):7.3f}",
          flush=True)


if __name__ == "__main__":
    main()
