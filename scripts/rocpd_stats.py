#!/usr/bin/env python
"""Per-kernel count / average / total from a rocprofv3 SQLite output (rocpd *.db), longest total first.
    python scripts/rocpd_stats.py <dir-or-db> [--top 20] [--match substr]"""
import argparse
import glob
import os
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    db = a.path if a.path.endswith(".db") else sorted(glob.glob(os.path.join(a.path, "**", "*.db"), recursive=True))[0]
    c = sqlite3.connect(db)
    names = [r[0] for r in c.execute("select name from sqlite_master where type in ('table', 'view')")]
    kd = next(n for n in names if n.startswith("rocpd_kernel_dispatch"))
    ks = next(n for n in names if n.startswith("rocpd_info_kernel_symbol"))
    q = (f"select s.kernel_name, count(*), avg(d.end - d.start) / 1e3, sum(d.end - d.start) / 1e6 from {kd} d "
         f"join {ks} s on d.kernel_id = s.id group by s.kernel_name order by sum(d.end - d.start) desc")
    print("%-70s %6s %11s %10s" % ("kernel", "calls", "avg us", "total ms"))
    n = 0
    for name, cnt, avg, tot in c.execute(q):
        if a.match and a.match not in name:
            continue
        print("%-70s %6d %11.1f %10.2f" % (name[:70], cnt, avg, tot))
        n += 1
        if n >= a.top:
            break


if __name__ == "__main__":
    main()
