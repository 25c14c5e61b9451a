"""Per-kernel averages of SQ counters from several rocprofv3 --pmc passes.

  python tools/pmc_summary.py PREFIX     (reads PREFIX1, PREFIX2, ... directories)

Prints, per kernel name, every counter's mean per dispatch and the derived
ratios used in DESIGN.md: VALU instructions per MFMA, the fraction of wave
cycles spent waiting on issue (SQ_WAIT_INST_ANY) / parked (SQ_WAIT_ANY), and
MFMA-busy per wave cycle.  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count
quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES cycles (MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import sys


def main():
    prefix = sys.argv[1]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sorted(glob.glob(prefix + "*")):
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(vals.items(), key=lambda kv: -len(next(iter(kv[1].values())))):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        print(f"# {k[:150]}  ({n} dispatches)")
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:16.1f}")
        if m.get("SQ_INSTS_MFMA"):
            print(f"   VALU per MFMA                {m.get('SQ_INSTS_VALU', 0) / m['SQ_INSTS_MFMA']:16.2f}")
        if m.get("SQ_WAVE_CYCLES"):
            wc = m["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    print(f"   {c + ' / wave cycles':28s} {m[c] / wc:16.3f}")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m:
                print(f"   MFMA busy / SQ busy          {m['SQ_VALU_MFMA_BUSY_CYCLES'] / max(1.0, m['SQ_BUSY_CYCLES']):16.3f}")


if __name__ == "__main__":
    main()
