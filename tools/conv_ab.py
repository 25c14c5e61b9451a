"""A/B of the fp32 encoder conv kernels on the GPU: dr_encoder_features over
8192 synthetic 64x64 frames (one train_Agent epoch's warm-start frames at
B = 256, S = 64), per variant of the temporary DREAMER_CS_VARIANT switch;
prints ms per encode and checks the variants agree bitwise.  Run under
rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from dreamer_amd import Dreamer
    from dreamer_amd import _lib as L
    from dreamer_amd import hip
    from formula import FULL
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    d = Dreamer(dict(FULL), dev)
    wm = d.world_model
    dims = wm.dims(d.agent)
    enc = wm.packed()
    n = int(os.environ.get("CONV_AB_FRAMES", "8192"))
    g = torch.Generator().manual_seed(2)
    frames = torch.randint(0, 256, (n, 3, 64, 64), generator=g, dtype=torch.uint8).to(dev)
    starts = torch.arange(n, dtype=torch.int64, device=dev)
    fr = L.dr_frames(L.ptr(frames), n, L.ptr(starts), None, 0, 0, 1, 0)
    feat = torch.empty(n, dims.enc_hidden, device=dev)
    ws = torch.empty(L.query("dr_encoder_workspace_bytes", dims, n), dtype=torch.uint8, device=dev)
    ref = None
    for var in sys.argv[1:] or ["0"]:
        os.environ["DREAMER_CS_VARIANT"] = var
        run = lambda: L.call("dr_encoder_features", dims, enc, fr, n, 1, L.ptr(feat), L.ptr(ws), ws.numel(),
                             hip.stream())
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        t = time.perf_counter()
        reps = 10
        for _ in range(reps):
            run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3 / reps
        out = feat.clone()
        same = None if ref is None else bool(torch.equal(out, ref))
        maxd = None if ref is None else float((out - ref).abs().max())
        ref = out if ref is None else ref
        print(f"variant {var}: {ms:.3f} ms per encode of {n} frames; bitwise equal to first: {same} (max diff {maxd})",
              flush=True)


if __name__ == "__main__":
    main()
