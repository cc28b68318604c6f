"""Derive per-kernel execution metrics from one rocprofv3 --pmc pass (developer tool).

Counters expected in the pass (8 SQ + 1 GRBM slots):
  SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
Derivations (MI355X_MICROARCH.md §rocprofv3 PMC slots, §Per-instruction cycle constants, 'DVFS give-back'):
  clock        = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration
  mfma_busy    = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x clock x duration)   (counts cycles: 16 per 16x16x32 bf16)
  issue split  = SQ_ACTIVE_INST_ANY / SQ_WAIT_INST_ANY / SQ_WAIT_ANY as fractions of SQ_WAVE_CYCLES (disjoint;
                 quad-cycle units, the ratio is unit-free): issuing / issue-stalled (dependency, pipe busy) / parked
                 (s_waitcnt, barrier)
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
Usage: python tools/sq_derive.py gpurun_out/<dir>/pmc_counter_collection.csv [kernel-substring] [--json out.json]
       (or the rocpd SQLite database rocprofv3 writes by default: gpurun_out/<dir>/<name>_results.db)
"""
import collections
import csv
import json
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    if out_json in args:
        args.remove(out_json)
    path = args[0]
    sub = args[1] if len(args) > 1 else "hiseg"
    if path.endswith(".db"):
        import sqlite3
        cur = sqlite3.connect(path).cursor()
        cur.execute("select dispatch_id, kernel_name, counter_name, value, start, end from counters_collection")
        rows = [{"Dispatch_Id": str(r[0]), "Kernel_Name": r[1], "Counter_Name": r[2], "Counter_Value": r[3],
                 "Start_Timestamp": r[4], "End_Timestamp": r[5]} for r in cur.fetchall()]
    else:
        rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    name = {}
    for r in rows:
        if sub not in r["Kernel_Name"]:
            continue
        did = r["Dispatch_Id"]
        per[did][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        name[did] = r["Kernel_Name"].split("(")[0]
    by_kernel = collections.defaultdict(list)
    for did in per:
        by_kernel[name[did]].append(did)
    result = {}
    for k, dids in by_kernel.items():
        c = collections.defaultdict(float)
        t = 0.0
        for did in dids:
            for n, v in per[did].items():
                c[n] += v
            t += dur[did]
        n = len(dids)
        m = {"dispatches": n, "avg_us": round(t / n * 1e6, 1)}
        if c.get("GRBM_GUI_ACTIVE"):
            clk = c["GRBM_GUI_ACTIVE"] / 8 / t
            m["clock_ghz"] = round(clk / 1e9, 3)
            if c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
                m["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * clk * t), 4)
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            m["issuing"] = round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4)
            m["issue_stalled"] = round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
            m["parked"] = round(c.get("SQ_WAIT_ANY", 0) / wc, 4)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            m["lds_conflict"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 4)
        m["raw_per_dispatch"] = {n2: round(v / n, 1) for n2, v in sorted(c.items())}
        result[k] = m
        print(k[:100])
        print("   ", {a: b for a, b in m.items() if a != "raw_per_dispatch"})
    if out_json:
        with open(out_json, "w") as f:
            json.dump(result, f, indent=1)


if __name__ == "__main__":
    main()
