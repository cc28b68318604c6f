"""Measured HBM bytes and bandwidth per kernel class from two rocprofv3 PMC passes (developer tool).

Pass 1: rocprofv3 --pmc FETCH_SIZE --kernel-trace -d <dir_f> -o pmc --output-format csv -- <cmd>
Pass 2: the same with --pmc WRITE_SIZE into <dir_w>.
HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) KiB (gfx950 correction, MI355X_MICROARCH.md §HBM; the same
rule as tools/pmc_summary.py).  Launches are grouped by kernel name and grid size; each group reports launches,
average duration (pass 1), average HBM MB per launch and the resulting GB/s.  Sorted by total time.
Usage: python tools/pmc_hbm.py <dir_f> <dir_w> [--top 30] [--match substring]
"""
import collections
import csv
import sys


def load(d, counter):
    out = {}
    for r in csv.DictReader(open(f"{d}/pmc_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        key = (r["Kernel_Name"].replace("void ", "").replace("hiseg::", "").split("(")[0][:90], int(r["Grid_Size"]))
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        out.setdefault(key, []).append((float(r["Counter_Value"]), dur))
    return out


def main():
    df, dw = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 30
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
    f, w = load(df, "FETCH_SIZE"), load(dw, "WRITE_SIZE")
    rows = []
    for key, fv in f.items():
        if match not in key[0] or key not in w:
            continue
        wv = w[key]
        n = min(len(fv), len(wv))
        fetch = sum(v for v, _ in fv[:n]) / n
        write = sum(v for v, _ in wv[:n]) / n
        dur = sum(d for _, d in fv[:n]) / n
        hbm = (2 * fetch + write) * 1024
        rows.append((dur * n, key, n, dur, hbm))
    print(f"{'launches':>8} {'avg_us':>8} {'HBM_MB':>9} {'GB/s':>7}  grid  kernel")
    for _, key, n, dur, hbm in sorted(rows, reverse=True)[:top]:
        print(f"{n:8d} {dur / 1e3:8.1f} {hbm / 1e6:9.1f} {hbm / dur:7.0f}  {key[1]:>9}  {key[0]}")


if __name__ == "__main__":
    main()
