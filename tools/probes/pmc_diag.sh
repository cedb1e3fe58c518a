#!/bin/bash
# GPU-box: diagnostic PMC passes of the joint step (one engine call), one rocprofv3 run per pass,
# each under its own time limit; the chain stops at the first failure.  FSEM_LIB selects the
# library.  Usage: bash tools/probes/pmc_diag.sh TAG
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${1:-pd}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
while read -r COUNTERS; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $COUNTERS -d $OUT/pmc_diag$i -o run --output-format csv -- python $R/tools/one_step.py --reps 1 --joint > $OUT/pmc_diag$i.log 2>&1 || { echo "PASS $i FAILED ($COUNTERS)"; tail -5 $OUT/pmc_diag$i.log; exit 1; }
  echo "pass $i ok: $COUNTERS"
done <<'LIST'
SQ_INSTS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE
SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE
SQC_DCACHE_MISSES SQC_DCACHE_HITS SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
LIST
cd $R && python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + "/pmc_diag*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fsem" in r["Kernel_Name"]:
            acc[r["Kernel_Name"].split("(")[0].replace("void ", "")][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    print(k)
    for c in sorted(v):
        print(f"   {c:28s} {v[c]:16.0f}")
PY
