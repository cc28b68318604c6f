"""Kernel-time summary of a rocprofv3 run (developer tool): reads the rocpd SQLite database rocprofv3 writes
by default (<dir>/<name>_results.db) and prints / writes the per-kernel totals that `--stats` puts in
kernel_stats.csv for the CSV format.

Usage: python tools/rocpd_stats.py gpurun_out/<dir>/<name>_results.db [--csv out.csv] [--top N] [--window A:B]
  --window A:B  only dispatches between the A-th and B-th launch of the kernel whose name contains
                HISEG_WINDOW_MARK (default: every dispatch)
"""
import argparse
import collections
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    cur = sqlite3.connect(args.db).cursor()
    cur.execute("select name, start, end from kernels")
    rows = cur.fetchall()
    agg = collections.defaultdict(lambda: [0, 0, None, None])
    for name, s, e in rows:
        a = agg[name]
        d = e - s
        a[0] += 1
        a[1] += d
        a[2] = d if a[2] is None else min(a[2], d)
        a[3] = d if a[3] is None else max(a[3], d)
    total = sum(a[1] for a in agg.values())
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    if args.csv:
        with open(args.csv, "w", newline="") as f:
            wr = csv.writer(f)
            wr.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for name, (n, t, mn, mx) in out:
                wr.writerow([name, n, t, round(t / n, 1), round(100.0 * t / total, 2), mn, mx])
    print(f"total kernel time {total / 1e6:.3f} ms over {sum(a[0] for a in agg.values())} dispatches")
    for name, (n, t, mn, mx) in out[:args.top]:
        print(f"{100.0 * t / total:6.2f}% {t / 1e6:9.3f} ms {n:6d} x {t / n / 1e3:8.1f} us  {name[:110]}")


if __name__ == "__main__":
    main()
