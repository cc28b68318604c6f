"""Measured HBM bytes per train / distill step for each kernel class of bench.call_profile, from two rocprofv3 PMC
passes over the same command (developer tool).

Pass 1: rocprofv3 --pmc FETCH_SIZE --kernel-trace -d <dir_f> -o pmc --output-format csv -- <cmd>
Pass 2: the same with --pmc WRITE_SIZE into <dir_w>.
HBM bytes per dispatch = (2 * FETCH_SIZE + WRITE_SIZE) KiB (the gfx950 correction of MI355X_MICROARCH.md, as in
tools/pmc_hbm.py).  Dispatches map to classes by kernel name; steps are counted by the optimizer's commit kernel.
The two passes must run the same command (same dispatch sequence); dispatches are matched by their index in
Dispatch_Id order (round 5: start-time order differed between passes where two streams interleave).

Usage: python tools/pmc_classes.py <dir_f> <dir_w> [--step-kernel adamw_seg_commit] [--json out.json --leg NAME]
"""
import argparse
import csv
import json
import re

CLASSES = [   # (class name as in bench.call_profile, kernel-name pattern); first match wins
    ("conv weight gradient", r"wgrad"),
    ("BatchNorm (train)", r"\bbn_|bn_stats|bn_apply|bn_bwd|bn_finalize"),
    ("depthwise conv (+ SE pool)", r"dwconv"),
    ("conv forward + data gradient", r"conv_(hwc|hwr|hwt|hw|fast|wide|igemm|pw|small|rows|splitk_reduce)"),
]


def load(d, counter):
    rows = [r for r in csv.DictReader(open(f"{d}/pmc_counter_collection.csv")) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))   # host enqueue order: the same in both passes with two streams
    return [(r["Kernel_Name"], float(r["Counter_Value"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            for r in rows]


def classify(name):
    for cls, pat in CLASSES:
        if re.search(pat, name):
            return cls
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir_f")
    ap.add_argument("dir_w")
    ap.add_argument("--step-kernel", default="adamw_seg_commit")
    ap.add_argument("--json")
    ap.add_argument("--leg", default="train")
    a = ap.parse_args()
    f, w = load(a.dir_f, "FETCH_SIZE"), load(a.dir_w, "WRITE_SIZE")
    n = min(len(f), len(w))
    if len(f) != len(w):
        print(f"warning: {len(f)} FETCH dispatches vs {len(w)} WRITE dispatches; matching the first {n}")
    steps = sum(1 for name, _, _ in f[:n] if a.step_kernel in name)
    if steps == 0:
        raise SystemExit(f"no '{a.step_kernel}' dispatch: cannot count steps")
    tot = {}
    for (nf, vf, df), (nw, vw, _) in zip(f[:n], w[:n]):
        if nf != nw and classify(nf) != classify(nw):
            # (a placement-dependent kernel choice, e.g. the weight gradient's transposed-read vs register-transpose
            # form, may differ between the passes; the class must not)
            raise SystemExit(f"dispatch sequences differ: {nf[:60]} vs {nw[:60]}")
        c = tot.setdefault(classify(nf), [0.0, 0.0, 0])
        c[0] += (2 * vf + vw) * 1024
        c[1] += df
        c[2] += 1
    out = {}
    for cls, (b, dur, cnt) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        out[cls] = {"hbm_bytes_per_step": b / steps, "kernel_ms_per_step": dur / steps / 1e6,
                    "dispatches_per_step": cnt / steps, "measured_gbs": b / dur if dur else None}
        print(f"{cls:32s} {b / steps / 1e9:8.3f} GB/step  {dur / steps / 1e6:8.3f} ms/step  "
              f"{cnt / steps:6.0f} dispatches/step  {b / dur if dur else 0:8.1f} GB/s")
    print(f"({steps} steps counted by '{a.step_kernel}')")
    if a.json:
        try:
            doc = json.load(open(a.json))
        except (OSError, ValueError):
            doc = {}
        doc.setdefault("train_legs", {})[a.leg] = out
        json.dump(doc, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
