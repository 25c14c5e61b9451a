"""Summarise two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) per kernel.

FETCH_SIZE is doubled: on gfx950 it reports half the bytes of wide coalesced
reads (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is taken as is.  Both
count L2 memory-side (fabric) requests, Infinity-Cache hits included.
Writes profiles-style text to stdout and a JSON with the encoder group's
per-epoch traffic when `--json PATH` is given.
"""
import collections
import csv
import glob
import json
import sys

ENCODER = ("k_enc12_split3", "k_conv_split3", "k_conv_glds_s3", "k_conv_glds_bf16", "k_conv_nhwc", "k_frames_nhwc4", "k_conv1_direct", "k_conv1_frames", "k_enc12_bf16", "k_conv_bf16", "k_conv1_bf16")


def load(d, counter):
    per = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    fe, wr = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    rows = []
    for k in set(fe) | set(wr):
        n = max(len(fe.get(k, [])), len(wr.get(k, [])))
        fb = 2.0 * 1024 * sum(fe.get(k, [])) / max(1, len(fe.get(k, [])))  # KB -> bytes, x2 gfx950
        wb = 1024 * sum(wr.get(k, [])) / max(1, len(wr.get(k, [])))
        rows.append((fb + wb, fb, wb, n, k))
    rows.sort(reverse=True)
    print("# per-dispatch HBM-side bytes (FETCH_SIZE x2 + WRITE_SIZE), rocprofv3 --pmc, separate passes")
    print("#   MB/dispatch   read MB   write MB  dispatches  kernel")
    for tot, fb, wb, n, k in rows[:40]:
        print(f"{tot / 1e6:14.3f} {fb / 1e6:9.3f} {wb / 1e6:9.3f} {n:10d}  {k[:110]}")
    enc = [(tot, n, k) for tot, fb, wb, n, k in rows if any(e in k for e in ENCODER)]
    enc_bytes = sum(t for t, n, k in enc)  # one dispatch of each per epoch
    print(f"# encoder group (conv stack + frame conversion; the feature-projection GEMM excluded), bytes per epoch: {enc_bytes:.0f}")
    if out_json:
        json.dump({"encoder_bytes_per_epoch": enc_bytes, "kernels": {k: t for t, n, k in enc},
                   "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, FETCH_SIZE x2 (gfx950)"},
                  open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main()
