"""Summary of tools/ab_trace.sh: per variant, the median duration (ms) of each engine kernel and
of the joint step over every traced call after the first two of each process.

    python tools/ab_trace_summary.py gpurun_out/TAG VAR...
"""
import csv
import glob
import os
import re
import statistics
import sys

KERNELS = ("pesq_front<true", "stoi_select", "stoi_tob", "stoi_seg(", "pesq_back", "stoi_seg_sum")


def calls(path):
    """Engine kernels of one trace, grouped per joint call (a call starts at pesq_front<true)."""
    f = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        return []
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
    out, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "fsem::" not in name:
            continue
        if "pesq_front<true" in name:
            cur = []
            out.append(cur)
        if cur is not None:
            cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return out


def main():
    base, variants = sys.argv[1], sys.argv[2:]
    res = {}
    for v in variants:
        per = {k: [] for k in KERNELS}
        steps = []
        for d in sorted(glob.glob(os.path.join(base, f"tr_{v}_*"))):
            if not os.path.isdir(d):
                continue
            for c in calls(d)[2:]:
                for k in KERNELS:
                    ds = [(e - s) / 1e6 for n, s, e in c if k in n]
                    if ds:
                        per[k].append(sum(ds))
                steps.append((max(e for _, _, e in c) - min(s for _, s, _ in c)) / 1e6)
        res[v] = (per, steps)
    head = "variant".ljust(10) + "".join(re.sub(r"[<(]$", "", k).ljust(14) for k in KERNELS) + "step"
    print(head)
    for v, (per, steps) in res.items():
        line = v.ljust(10)
        for k in KERNELS:
            line += (f"{statistics.median(per[k]):.4f}" if per[k] else "-").ljust(14)
        line += f"{statistics.median(steps):.4f}" if steps else "-"
        print(line + f"   ({len(steps)} calls)")


if __name__ == "__main__":
    main()
