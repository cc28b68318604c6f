"""Per-kernel instruction-cache misses from one rocprofv3 PMC pass (developer tool; CPU-side summary).

    rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES --kernel-trace --output-format csv -d D -o pmc -- \
        python3 bench.py --leg distill --eager-train --steps 2 --warmup 1
    python tools/pmc_icache.py D

Prints, per kernel name (summed over its dispatches): dispatches, average duration (kernel trace), instruction-cache
misses per dispatch and per wave, and the miss share -- kernels whose short launches are paid in instruction fetch
(tools/icache_probe.hip) show many misses per wave at small durations.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in cc:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    dur = defaultdict(list)
    for f in kt:
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for k, c in per.items():
        n = len(disp[k])
        miss, hit, waves = c.get("SQC_ICACHE_MISSES", 0.0), c.get("SQC_ICACHE_HITS", 0.0), c.get("SQ_WAVES", 0.0)
        us = sum(dur[k]) / len(dur[k]) if dur[k] else float("nan")
        rows.append((miss, n, us, miss / max(n, 1), miss / max(waves, 1), miss / max(miss + hit, 1), k[:110]))
    rows.sort(reverse=True)
    print(f"{'misses':>10} {'disp':>5} {'avg_us':>8} {'miss/disp':>10} {'miss/wave':>9} {'miss%':>6}  kernel")
    for r in rows[:60]:
        print(f"{r[0]:10.0f} {r[1]:5d} {r[2]:8.1f} {r[3]:10.0f} {r[4]:9.2f} {100 * r[5]:6.1f}  {r[6]}")


if __name__ == "__main__":
    main(sys.argv[1])
