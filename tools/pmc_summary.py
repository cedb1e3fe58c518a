"""Per-kernel PMC summary of a tools/gpu_round.sh run (separate rocprofv3 --pmc passes).

    python tools/pmc_summary.py gpurun_out/<tag> > profiles/<round>/pmc_summary.json

Per fsem kernel, averaged over its launches: raw counter values, plus HBM bytes corrected as
MI355X_MICROARCH.md 'HBM' prescribes: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE counts half the bytes of wide (16 B/lane) coalesced streaming reads, so
hbm_read_bytes = 2 * 1024 * FETCH_SIZE; hbm_write_bytes = 1024 * WRITE_SIZE.  "_meta" records the
rows and length of one profiled engine call (env PMC_ROWS / PMC_LENGTH, set by the drivers) and
the build id of the profiled library; bench.py only takes counters recorded on its own library
build at its own per-launch size.
"""
import collections
import csv
import glob
import json
import os
import sys


def short(name: str) -> str:
    base = name.split("(")[0].replace("void ", "")
    return base


def main(root: str):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "fsem" not in r["Kernel_Name"]:
                continue
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, counters in acc.items():
        d = {c: sum(v) / len(v) for c, v in counters.items()}
        d["launches"] = max(len(v) for v in counters.values())
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes"] = 2 * 1024 * d["FETCH_SIZE"]
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = 1024 * d["WRITE_SIZE"]
        if "hbm_read_bytes" in d and "hbm_write_bytes" in d:
            d["hbm_bytes"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
        if "SQ_WAVE_CYCLES" in d and d.get("GRBM_GUI_ACTIVE"):
            # mean resident waves per SIMD over the launch: SQ_WAVE_CYCLES counts quad-cycles
            # (x4), GRBM_GUI_ACTIVE is summed over the 8 XCDs (/8 = the launch's cycles), and
            # the chip has 256 CUs x 4 SIMDs (tools/gpu_round.sh collects both in its SQ pass).
            d["waves_per_simd"] = 4 * d["SQ_WAVE_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8 * 1024)
        out[k] = d
    # the engine call the passes profiled (tools/one_step.py: the drop-in call's row chunk)
    # and the library build it ran (fsem_build_id, read from the file the passes loaded: FSEM_LIB
    # or the in-tree libfsem.so): bench.py takes counters of its own build and size only
    sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
    from fast_speech_enhancement_metrics_amd import _build
    lib = os.environ.get("FSEM_LIB", _build.LIB)
    out["_meta"] = {"rows_per_launch": int(os.environ.get("PMC_ROWS", "4096")),
                    "length": int(os.environ.get("PMC_LENGTH", "160000")),
                    "build_id": _build.library_build_id(lib), "library": os.path.basename(lib)}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
