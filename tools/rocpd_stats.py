"""Kernel (and HIP API) statistics from a rocprofv3 rocpd SQLite database
(the .db a `rocprofv3 --kernel-trace/--runtime-trace` run writes): name,
calls, total / average / min / max ns -- the columns of rocprofv3's
kernel_stats.csv. Usage: python tools/rocpd_stats.py DB [--api] [--csv OUT]."""
import argparse
import csv
import sqlite3
import sys


def kernel_stats(db):
    con = sqlite3.connect(db)
    rows = con.execute(
        "select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end - d.start), "
        "max(d.end - d.start) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
        "group by s.kernel_name order by sum(d.end - d.start) desc").fetchall()
    return rows


def api_stats(db):
    con = sqlite3.connect(db)
    rows = con.execute(
        "select n.string, count(*), sum(r.end - r.start), avg(r.end - r.start), min(r.end - r.start), "
        "max(r.end - r.start) from rocpd_region r join rocpd_string n on r.name_id = n.id "
        "group by n.string order by sum(r.end - r.start) desc").fetchall()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--api", action="store_true")
    ap.add_argument("--csv")
    a = ap.parse_args()
    rows = api_stats(a.db) if a.api else kernel_stats(a.db)
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"]
    out = open(a.csv, "w", newline="") if a.csv else sys.stdout
    w = csv.writer(out)
    w.writerow(hdr)
    for r in rows:
        w.writerow([r[0], r[1], r[2], round(r[3], 1), r[4], r[5]])


if __name__ == "__main__":
    main()
