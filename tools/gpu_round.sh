#!/bin/bash
# GPU-box driver: parity tests, bench, kernel trace + PMC passes. Each GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
R=$PWD
TAG=${1:-r}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python $R/tools/one_step.py --reps 3 --joint > $OUT/trace.log 2>&1 || { echo "TRACE FAILED"; tail -20 $OUT/trace.log; exit 1; }
if [ "${PMC:-1}" = "1" ]; then
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python $R/tools/one_step.py --reps 1 --joint > $OUT/pmc1.log 2>&1 || { echo "PMC1 FAILED"; tail -20 $OUT/pmc1.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python $R/tools/one_step.py --reps 1 --joint > $OUT/pmc2.log 2>&1 || { echo "PMC2 FAILED"; tail -20 $OUT/pmc2.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o run --output-format csv -- python $R/tools/one_step.py --reps 1 --joint > $OUT/pmc3.log 2>&1 || { echo "PMC3 FAILED"; tail -20 $OUT/pmc3.log; exit 1; }
fi
echo DONE
