#!/bin/bash
# One PMC pass for LDS-pipe utilisation per kernel: SQ_LDS_IDX_ACTIVE (all LDS-array cycles),
# bank conflicts, LDS instructions, against GRBM_GUI_ACTIVE (GPU busy cycles).
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${1:-pl}; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_lds -o run --output-format csv -- python $R/tools/one_step.py --reps 1 "$@" > $OUT/pmc.log 2>&1 || { echo "PMC FAILED"; tail -20 $OUT/pmc.log; exit 1; }
python3 $R/tools/pmc_lds_summary.py $OUT
