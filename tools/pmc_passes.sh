#!/bin/bash
# GPU-box: the three PMC passes of tools/gpu_round.sh alone (one_step.py --joint, one engine call
# of 4096 x 10 s per pass) and their summary.  Usage: bash tools/pmc_passes.sh TAG
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${1:-pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python $R/tools/one_step.py --reps 1 --joint > $OUT/pmc1.log 2>&1 || { echo "PMC1 FAILED"; tail -20 $OUT/pmc1.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python $R/tools/one_step.py --reps 1 --joint > $OUT/pmc2.log 2>&1 || { echo "PMC2 FAILED"; tail -20 $OUT/pmc2.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY -d $OUT/pmc_sq -o run --output-format csv -- python $R/tools/one_step.py --reps 1 --joint > $OUT/pmc3.log 2>&1 || { echo "PMC3 FAILED"; tail -20 $OUT/pmc3.log; exit 1; }
cd $R && bash tools/pmc_lds.sh ${1:-pmc} --joint > $OUT/pmc_lds_valu.txt && PMC_ROWS=4096 python tools/pmc_summary.py $OUT > $OUT/pmc_summary.json && echo PMC_DONE
