"""Summarise a rocprofv3 kernel-trace database (prof_results.db) per kernel."""
import hashlib
import os
import sqlite3
import sys


def source_hash():
    """Content hash of the library sources (dreamer_amd/csrc, include): ties a
    profile summary to the tree it was measured on (bench.py compares it)."""
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    h = hashlib.sha256()
    for d in ("dreamer_amd/csrc", "include"):
        for f in sorted(os.listdir(os.path.join(root, d))):
            if f.endswith((".hip", ".h")):
                h.update(f.encode())
                h.update(open(os.path.join(root, d, f), "rb").read())
    return h.hexdigest()[:16]


def summary(db, top=40):
    con = sqlite3.connect(db)
    rows = con.execute("select name, count(*), sum(end-start), avg(end-start) from kernels group by name "
                       "order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    out = [f"# rocprofv3 --kernel-trace --stats summary of {db}", f"# source {source_hash()}",
           f"# total kernel time {tot/1e6:.3f} ms",
           "# total_ms  calls  avg_us  kernel"]
    for n, c, s, a in rows[:top]:
        out.append(f"{s/1e6:9.3f} {c:6d} {a/1e3:9.2f}  {n[:140]}")
    return "\n".join(out)


if __name__ == "__main__":
    print(summary(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40))
