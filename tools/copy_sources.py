"""Which HIP API calls launch the __amd_rocclr_copyBuffer kernels in a rocprofv3 trace (developer tool).
Usage: python tools/copy_sources.py <dir with *_kernel_trace.csv and *_hip_api_trace.csv>"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
at = glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True)[0]
api = {}
for r in csv.DictReader(open(at)):
    api[r["Correlation_Id"]] = r["Function"]
cnt = collections.Counter()
dur = collections.Counter()
for r in csv.DictReader(open(kt)):
    if "copyBuffer" in r["Kernel_Name"] or "fillBuffer" in r["Kernel_Name"]:
        k = (r["Kernel_Name"][:40], api.get(r["Correlation_Id"], "?"))
        cnt[k] += 1
        dur[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, c in cnt.most_common(20):
    print(c, round(dur[k] / 1e3, 1), "us", k)
