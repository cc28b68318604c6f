"""Per-kernel summary of the inference phase of a bench.py rocprofv3 kernel trace (developer tool).

bench.py runs the C2 inference leg first, then the train legs.  The kernel-stats CSV mixes them; this
keeps the launches before the first train-mode BatchNorm kernel (bn_stats) and, with --last-ms T, only
those that start in the last T ms before that cut (the timed steps), then groups them by kernel name and
grid size and prints total / average time, the share of the summed kernel time and the busy wall span.
--dominant N keeps the window from the first to the last of the N latest dominant-class launches
(conv_hwr_kernel / round-2 conv_hw_kernel<128> over 6144 workgroups: 9 per inference step).
Usage: python tools/phase_stats.py gpurun_out/<dir>/trace_kernel_trace.csv [--last-ms 250 | --dominant 45] [--top 40]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    last_ms = float(sys.argv[sys.argv.index("--last-ms") + 1]) if "--last-ms" in sys.argv else None
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    cut = next((int(r["Start_Timestamp"]) for r in rows if "bn_stats" in r["Kernel_Name"]), None)
    if cut is None:
        cut = int(rows[-1]["End_Timestamp"]) + 1
    rows = [r for r in rows if int(r["Start_Timestamp"]) < cut]
    if "--dominant" in sys.argv:   # window spanned by the last N launches of the dominant class (timed steps)
        nd = int(sys.argv[sys.argv.index("--dominant") + 1])
        dom = [r for r in rows if r["Kernel_Name"].startswith(("void hiseg::conv_hwr_kernel<", "void hiseg::conv_hw_kernel<128"))
               and int(r["Grid_Size_X"]) == 6144 * 256][-nd:]
        t0, t1 = int(dom[0]["Start_Timestamp"]), int(dom[-1]["End_Timestamp"])
        rows = [r for r in rows if t0 <= int(r["Start_Timestamp"]) <= t1]
    if last_ms is not None:
        t0 = max(int(r["End_Timestamp"]) for r in rows) - int(last_ms * 1e6)
        rows = [r for r in rows if int(r["Start_Timestamp"]) >= t0]
    groups = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        name = name[5:] if name.startswith("void ") else name
        groups[(name[:90], int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    total = sum(sum(v) for v in groups.values())
    span = (max(int(r["End_Timestamp"]) for r in rows) - min(int(r["Start_Timestamp"]) for r in rows)) / 1e3
    print(f"launches {len(rows)}  summed kernel time {total / 1e3:.2f} ms  wall span {span / 1e3:.2f} ms")
    print(f"{'share':>6} {'total_ms':>9} {'calls':>6} {'avg_us':>8}  grid  kernel")
    for (name, grid), v in sorted(groups.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print(f"{100 * sum(v) / total:5.1f}% {sum(v) / 1e3:9.3f} {len(v):6d} {sum(v) / len(v):8.1f}  {grid:>9}  {name}")


if __name__ == "__main__":
    main()
