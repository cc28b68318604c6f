"""Per-step GPU busy time vs wall time from a rocprofv3 kernel trace (developer tool): steps are delimited by the
launches of a marker kernel (one per step, e.g. the fused AdamW); busy = union of kernel intervals in the step.

Usage: python tools/step_gaps.py <results.db> [--marker adamw] [--last 10]"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="adamw")
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    cur.execute("select name, start, end from kernels order by start")
    rows = cur.fetchall()
    marks = [i for i, (n, s, e) in enumerate(rows) if a.marker in n.lower()]
    if len(marks) < 2:
        raise SystemExit(f"marker '{a.marker}' found {len(marks)} times")
    marks = marks[-(a.last + 1):]
    walls, busys, counts = [], [], []
    per = collections.defaultdict(float)
    for m0, m1 in zip(marks, marks[1:]):
        seg = rows[m0 + 1:m1 + 1]
        t0, t1 = rows[m0][2], rows[m1][2]
        busy, cur_s, cur_e = 0, None, None
        for n, s, e in seg:
            per[n] += (e - s)
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        walls.append(t1 - t0)
        busys.append(busy)
        counts.append(len(seg))
    k = len(walls)
    print(f"{k} steps: wall {sum(walls) / k / 1e6:.3f} ms, GPU busy {sum(busys) / k / 1e6:.3f} ms "
          f"({sum(busys) / sum(walls):.3f}), kernels per step {sum(counts) / k:.0f}, "
          f"idle per kernel {(sum(walls) - sum(busys)) / sum(counts) / 1e3:.2f} us")
    tot = sum(per.values())
    for n, v in sorted(per.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"  {100 * v / tot:5.1f}%  {v / k / 1e6:7.3f} ms/step  {n[:110]}")


if __name__ == "__main__":
    main()
