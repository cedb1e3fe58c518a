#!/bin/bash
# One PMC pass for LDS-pipe utilisation per kernel: SQ_LDS_IDX_ACTIVE (all LDS-array cycles),
# bank conflicts, LDS instructions, against GRBM_GUI_ACTIVE (GPU busy cycles).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${1:-pl}; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_lds -o run --output-format csv -- python $R/tools/one_step.py --reps 1 "$@" > $OUT/pmc.log 2>&1 || { echo "PMC FAILED"; tail -20 $OUT/pmc.log; exit 1; }
python3 - $OUT <<'PY'
import collections, csv, glob, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/pmc_lds/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fsem" in r["Kernel_Name"]:
            acc[r["Kernel_Name"].split("(")[0][:44]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    g = max(v["GRBM_GUI_ACTIVE"], 1)
    print(f"{k:44s} gui {g:12.0f} lds_idx_active/cu/gui {v['SQ_LDS_IDX_ACTIVE'] / 256 / g:6.3f} "
          f"conf/cu/gui {v['SQ_LDS_BANK_CONFLICT'] / 256 / g:6.3f} valu/simd/gui {v['SQ_INSTS_VALU'] * 4 / 1024 / g:6.3f} "
          f"busy {v['SQ_BUSY_CYCLES'] / g:6.3f}  " + " ".join(f"{c}={x:.3g}" for c, x in v.items()))
PY
