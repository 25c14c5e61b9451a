"""Per-kernel SQ / TCC counter summary of tools/pmc_sq.sh's two rocprofv3 passes.

Prints, per kernel (averaged over its dispatches): waves, VALU and MFMA
instructions per wave, the split of wave cycles into issue-waits
(SQ_WAIT_INST_ANY), other waits (SQ_WAIT_ANY: s_waitcnt / barrier) and
active issue (SQ_ACTIVE_INST_ANY), and the L2 hit rate.
"""
import collections
import csv
import glob
import sys

KEYS = ("k_gemm_wks3", "k_gru_gates", "k_ln_gemm_sample", "k_gru_fused", "k_pscan", "k_pdream", "k_gemm_skinny",
        "k_enc12", "k_conv_split3", "k_conv_bf16", "k_actor_head_bwd_x", "k_zgather_add", "k_mlp2_tail",
        # world-model step kernels
        "k_convT", "k_wgrad", "k_conv_wgrad", "k_conv_nhwc", "k_gemm_tile", "k_gemm_pp_multi", "k_kn_repack",
        "k_gemm_wk<", "k_conv_glds", "k_gemm_glds")


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    print("# rocprofv3 --pmc, two passes (SQ; TCC + GRBM), per dispatch averages")
    print("# disp  waves  valu/wave  mfma/wave  wait_inst  wait_any  active   L2hit  kernel")
    rows = []
    for k, c in a.items():
        if not any(x in k for x in KEYS):
            continue
        avg = lambda d, n: sum(d.get(n, [0])) / max(1, len(d.get(n, [])))
        w = avg(c, "SQ_WAVES")
        cyc = avg(c, "SQ_WAVE_CYCLES") or 1.0
        hit, miss = avg(b.get(k, {}), "TCC_HIT_sum"), avg(b.get(k, {}), "TCC_MISS_sum")
        rows.append((len(c.get("SQ_WAVES", [])), w, avg(c, "SQ_INSTS_VALU") / max(w, 1), avg(c, "SQ_INSTS_MFMA") / max(w, 1),
                     avg(c, "SQ_WAIT_INST_ANY") / cyc, avg(c, "SQ_WAIT_ANY") / cyc, avg(c, "SQ_ACTIVE_INST_ANY") / cyc,
                     hit / max(hit + miss, 1), k))
    rows.sort(key=lambda r: -r[0])
    for n, w, v, m, wi, wa, ac, h, k in rows:
        print(f"{n:6d} {w:6.0f} {v:10.1f} {m:10.1f} {wi:10.3f} {wa:9.3f} {ac:7.3f} {h:7.3f}  {k[:100]}")


if __name__ == "__main__":
    main()
