"""Average duration of bench.py's dominant launch class from a rocprofv3 kernel trace (developer tool).

The dominant class is the 256->256 3x3 conv at the 64x48 ROI grid over 256 ROIs.  Round 3: conv_hwr_kernel
(6144 workgroups of 256, default); round 2: conv_hw_kernel<128> (--hw), before it the wide-tile
kernel conv_wide_kernel<256, 4, ...> with 3072 pixel tiles x 1 Cout tile (grid 786 432 threads: 256-thread
workgroups); round 1: conv_fast_kernel<128, 128, ...>, 12288 workgroups of 512 (--r1).  The kernel-stats
summary averages every launch of a kernel (all layer shapes); this filters the trace to the class bench.py's
HIP-event probe times, so the two averages can be compared.  The same grid also runs the 128->256 3x3
(K = 1152) layer; the trace carries no shape, so the K = 2304 class is taken as the launches longer than 0.55 (r1: 0.75) x the median of the upper half (the K values are
2x apart; with the 2-stream schedule a launch overlapped by the next step's UNet stretches up to 2x, hence
the lower cut).
The bench's probe times the inference launches only; the trace of a full bench run also holds the same
class from the train step (uncontended: no UNet overlapping it), so launches from the first training kernel
on (bn_stats: train-mode BatchNorm) are dropped, and with --last N only the N latest inference launches
(the timed steps: 9 per step) are kept.
Usage: python tools/dominant_from_trace.py gpurun_out/prof_v5/trace_kernel_trace.csv [--last N] > profiles/...json
"""
import csv
import json
import sys

R1 = "--r1" in sys.argv
WIDE = "--wide" in sys.argv    # round 2 v1: conv_wide_kernel<256, 4>
GRID = 12288 * 512 if R1 else (3072 * 256 if WIDE else 6144 * 256)
HW = "--hw" in sys.argv        # round 2 v2-v12: conv_hw_kernel<128, ...>
HWR = "--hwr" in sys.argv      # rounds 3-4: conv_hwr_kernel; default (round 5): conv_hwc_kernel (same grid)
PREFIX = ("void hiseg::conv_fast_kernel<128, 128" if R1 else
          "void hiseg::conv_wide_kernel<256, 4" if WIDE else
          "void hiseg::conv_hw_kernel<128" if HW else "void hiseg::conv_hwr_kernel<" if HWR else
          "void hiseg::conv_hwc_kernel<")
allrows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
cut_t = next((int(r["Start_Timestamp"]) for r in allrows if "bn_stats" in r["Kernel_Name"]), None)
rows = [r for r in allrows
        if r["Kernel_Name"].startswith(PREFIX) and int(r["Grid_Size_X"]) == GRID
        and (cut_t is None or int(r["Start_Timestamp"]) < cut_t)]
d_seq = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
d_all = sorted(d_seq)
upper = d_all[len(d_all) // 2:]
cut = (0.75 if R1 else 0.55) * upper[len(upper) // 2]
d = [v for v in d_seq if v > cut]
if "--last" in sys.argv:
    d = d[-int(sys.argv[sys.argv.index("--last") + 1]):]
d = sorted(d)
name = ("conv_fast_kernel<128,128,4,2,2,lds-epilogue> grid 12288 x 512" if R1 else
        "conv_wide_kernel<256,4> grid 3072 x 256" if WIDE else
        "conv_hw_kernel<128> grid 6144 x 256" if HW else "conv_hwr_kernel<ACT, RES, 6> grid 6144 x 256" if HWR else
        "conv_hwc_kernel<ACT, RES, 4> grid 6144 x 256")
print(json.dumps({"kernel": name + " (256->256 3x3 @64x48 x256 ROIs)",
                  "launches": len(d), "same_grid_launches": len(d_all), "cluster_cut_ms": round(cut, 4), "avg_ms": round(sum(d) / len(d), 4), "median_ms": round(d[len(d) // 2], 4),
                  "min_ms": round(d[0], 4), "max_ms": round(d[-1], 4),
                  "flop_per_launch": 927712935936.0,
                  "tflops_at_avg": round(927712935936.0 / (sum(d) / len(d) * 1e-3) / 1e12, 1)}, indent=1))
