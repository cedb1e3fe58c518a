#!/bin/bash
# GPU-box closing set of one library build (round 5 layout): GPU tests, the PMC passes of one
# joint engine call (HBM bytes, SQ counters, LDS activity) summarised into
# profiles/TAG/pmc_summary.json ON THE BOX (so the bench that follows finds the counters of
# its own build), the bench line, the bench under a kernel trace (+ per-step timeline), the
# other configurations' lines, and smoke().  Every GPU step has its own time limit; the chain
# stops at the first failure.  Usage: bash tools/r5_round.sh TAG [--no-tests]
set -o pipefail
R=$PWD
TAG=${1:-r5}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT $R/profiles/$TAG
if [ "${1:-}" != "--no-tests" ]; then
  bash tools/gpu_tests.sh $TAG || { echo "TESTS FAILED"; exit 1; }
fi
cd /tmp && export TMPDIR=/tmp
pmc() {  # pmc NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- python $R/tools/one_step.py --reps 1 --joint > $OUT/$name.log 2>&1 || { echo "PMC $name FAILED"; tail -20 $OUT/$name.log; exit 1; }
}
pmc pmc_fetch FETCH_SIZE
pmc pmc_write WRITE_SIZE
pmc pmc_sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE
pmc pmc_lds SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
cd $R
PMC_ROWS=4096 python tools/pmc_summary.py $OUT > $OUT/pmc_summary.json || exit 1
cp $OUT/pmc_summary.json $R/profiles/$TAG/pmc_summary.json
python tools/pmc_lds_summary.py $OUT > $OUT/pmc_lds_valu.txt 2>&1 || true
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/bench_trace.sh $TAG || exit 1
python tools/timeline.py $OUT/trace_bench > $OUT/timeline_bench.txt 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python $R/tools/one_step.py --reps 3 --joint > $OUT/trace.log 2>&1 || { echo "TRACE FAILED"; tail -20 $OUT/trace.log; exit 1; }
cd $R
for w in pesq c3 c5; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "BENCH $w FAILED"; exit 1; }
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail $OUT/smoke.txt; exit 1; }
cat $OUT/smoke.txt
echo ROUND_DONE
