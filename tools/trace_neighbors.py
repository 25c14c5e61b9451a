"""Launches around every call of one kernel in a rocprofv3 kernel-trace
database: the kernels just before / after it with durations (us), to find
which call site a kernel belongs to.
  python tools/trace_neighbors.py p_results.db <kernel-name-substring> [before] [after] [max_hits]"""
import sqlite3
import sys


def main():
    db, pat = sys.argv[1], sys.argv[2]
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    na = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    mx = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    hits = [i for i, r in enumerate(rows) if pat in r[0]]
    print(f"# {len(hits)} launches of '{pat}'")
    for i in hits[-mx:]:
        print("----")
        for j in range(max(0, i - nb), min(len(rows), i + na + 1)):
            n, s, e = rows[j]
            print(f"{'>>' if j == i else '  '} {(e - s) / 1e3:9.2f}  {n[:150]}")


if __name__ == "__main__":
    main()
