"""Per-epoch kernel table of a profiled bench run (rocprofv3 --kernel-trace).

  python tools/epoch_table.py prof_results.db EPOCHS ENCODES [top]

The profiled command is `bench.py --steps S --warmup W --no-cpu-baseline
--no-secondary --wm-steps 0`: EPOCHS = S + W train_Agent epochs, and the
encoder kernels run ENCODES = EPOCHS + 6 times (bench.py's live roofline timing
adds one warm-up and five timed encodes).  A kernel whose call count divides by
ENCODES but not by EPOCHS is counted as an encoder kernel.  Prints launches and
milliseconds per epoch, sorted by ms per epoch (the profiler serialises the
launches, so the sum is an upper bound of the replayed epoch)."""
import sqlite3
import sys


def main():
    db, epochs, encodes = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    con = sqlite3.connect(db)
    rows = con.execute("select name, count(*), sum(end-start), avg(end-start) from kernels group by name").fetchall()
    out = []
    for n, c, s, a in rows:
        per = encodes if (c % encodes == 0 and c % epochs != 0) else epochs
        out.append((s / per / 1e6, c / per, a / 1e3, n))
    out.sort(reverse=True)
    tot = sum(o[0] for o in out)
    print(f"# per-epoch kernel table of {db}: {epochs} epochs, {encodes} encoder runs; sum {tot:.3f} ms per epoch")
    print("# ms/epoch  launches/epoch  avg_us  kernel")
    for ms, calls, avg, n in out[:top]:
        print(f"{ms:9.4f} {calls:10.1f} {avg:9.2f}  {n[:130]}")


if __name__ == "__main__":
    main()
