"""Per-queue timeline of the last replayed step in a rocprofv3 kernel trace (developer tool).  Splits the trace
into steps at gaps > --gap-us between consecutive kernels, takes the last complete step and prints, per queue,
the kernel count, first start / last end relative to the step start and the busy time.
Usage: python tools/step_timeline.py <kernel_trace.csv> [--gap-us 40]"""
import csv
import sys


def main():
    path = sys.argv[1]
    gap = float(sys.argv[sys.argv.index("--gap-us") + 1]) if "--gap-us" in sys.argv else 40.0
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and s - last_end > gap * 1e3 and cur:
            steps.append(cur)
            cur = []
        cur.append(r)
        last_end = e if last_end is None else max(last_end, e)
    steps.append(cur)
    big = [st for st in steps if len(st) > 100]
    st = big[-2] if len(big) >= 2 else big[-1]
    t0 = int(st[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in st)
    print(f"steps found: {len(big)}; the one before last: {len(st)} kernels, {(t1 - t0) / 1e6:.3f} ms")
    byq = {}
    for r in st:
        byq.setdefault(r.get("Queue_Id"), []).append(r)
    for q, v in sorted(byq.items(), key=lambda kv: int(kv[1][0]["Start_Timestamp"])):
        s0 = min(int(r["Start_Timestamp"]) for r in v) - t0
        e1 = max(int(r["End_Timestamp"]) for r in v) - t0
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in v)
        print(f"  queue {q}: {len(v)} kernels, {s0 / 1e6:.3f} .. {e1 / 1e6:.3f} ms, kernel time {busy / 1e6:.3f} ms")
        top = {}
        for r in v:
            k = r["Kernel_Name"].split("(")[0][:70]
            top[k] = top.get(k, 0) + int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for k, t in sorted(top.items(), key=lambda kv: -kv[1])[:6]:
            print(f"      {t / 1e3:8.1f} us  {k}")


if __name__ == "__main__":
    main()
