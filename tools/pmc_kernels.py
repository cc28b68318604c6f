"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel (developer tool).
Usage: python tools/pmc_kernels.py gpurun_out/<dir>/pmc_counter_collection.csv [substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else "hiseg"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(set)
for r in rows:
    if sub not in r["Kernel_Name"]:
        continue
    k = r["Kernel_Name"].split("(")[0][:110]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur[k].add((r["Dispatch_Id"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
for k, c in agg.items():
    ds = [x[1] for x in dur[k]]
    print(k, f"dispatches={len(ds)} avg_us={sum(ds) / len(ds) / 1e3:.1f}")
    print("   ", {n: round(sum(v) / len(v) / 1e6, 3) for n, v in sorted(c.items())})
