"""Per-launch timeline of the engine's kernels from a rocprofv3 kernel_trace.csv:
offsets (ms) relative to each pesq_front start, to see overlap and gaps.

    python tools/timeline.py gpurun_out/TAG/trace
"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "fsem" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = None
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fsem::", "")
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "pesq_front" in name:
        t0 = s
        print("----")
    if t0 is None:
        continue
    print(f"{name:40s} q{r.get('Queue_Id', '?'):>3s} start {(s - t0) / 1e6:8.3f} end {(e - t0) / 1e6:8.3f} dur {(e - s) / 1e6:7.3f}")
