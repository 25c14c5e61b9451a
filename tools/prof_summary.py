"""Summarise a rocprofv3 kernel-trace database (prof_results.db) per kernel."""
import sqlite3
import sys


def summary(db, top=40):
    con = sqlite3.connect(db)
    rows = con.execute("select name, count(*), sum(end-start), avg(end-start) from kernels group by name "
                       "order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    out = [f"# rocprofv3 --kernel-trace --stats summary of {db}", f"# total kernel time {tot/1e6:.3f} ms",
           "# total_ms  calls  avg_us  kernel"]
    for n, c, s, a in rows[:top]:
        out.append(f"{s/1e6:9.3f} {c:6d} {a/1e3:9.2f}  {n[:140]}")
    return "\n".join(out)


if __name__ == "__main__":
    print(summary(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40))
