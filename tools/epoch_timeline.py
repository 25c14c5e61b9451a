"""Kernel timeline of one train_Agent epoch from a rocprofv3 kernel-trace
database: every launch of the epoch in order with its duration and the gap
to the previous kernel's end, grouped into the engine's phases by marker
kernels.  Usage: python tools/epoch_timeline.py p_results.db [epoch_index]

Epochs are delimited by the replay gather (k_replay_gather runs once per
train_Agent call, before the warm start)."""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if r[0].startswith("k_replay_gather")]
    if len(starts) < 2:
        print("no epochs found")
        return
    i0 = starts[which]
    i1 = starts[which + 1] if which + 1 < len(starts) and which != -1 else len(rows)
    ep = rows[i0:i1]
    t0 = ep[0][1]
    tot_k = sum(e - s for _, s, e in ep)
    print(f"# epoch {which}: {len(ep)} launches, wall {(ep[-1][2] - t0) / 1e3:.1f} us, kernel sum {tot_k / 1e3:.1f} us")
    agg = collections.OrderedDict()
    prev_end = t0
    for n, s, e in ep:
        short = n.split("(")[0][:60]
        gap = (s - prev_end) / 1e3
        prev_end = e
        a = agg.setdefault(short, [0, 0.0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e3
        a[2] += max(gap, 0.0)
    print("# launches  kernel_us  gaps_before_us  kernel")
    for k, (c, d, g) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{c:9d} {d:10.1f} {g:12.1f}  {k}")
    if len(sys.argv) > 3:
        prev_end = t0
        for n, s, e in ep:
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.2f} {(s - prev_end) / 1e3:6.2f}  {n.split('(')[0][:70]}")
            prev_end = e


if __name__ == "__main__":
    main()
