#!/bin/bash
# The round's closing measurement set of ONE library build, on the GPU box (one gpurun call):
#   1. the GPU test suite (tools/gpu_tests.sh)                          -> gpu_tests.log
#   2. PMC passes of one joint engine call at the bench's 4096 rows, one counter group per
#      rocprofv3 run (FETCH_SIZE, WRITE_SIZE, SQ issue / wait counters, LDS activity), summed
#      by tools/pmc_summary.py ON THE BOX into profiles/TAG/pmc_summary.json, so that the bench
#      line that follows finds the counters of its own build (bench.pmc_summary_for matches
#      build id, rows and length)                                       -> pmc_summary.json, pmc_lds_valu.txt
#   3. bench.py, the driver's command                                   -> bench.json
#   4. bench.py under rocprofv3 --kernel-trace --stats (its pesq_front average must agree with
#      the bench line's roofline.ms_per_launch) and the per-step timeline -> trace_bench/, timeline_bench.txt
#   5. the other configurations' lines (PESQ alone, config 3, config 5, PESQ with the three
#      time-alignment modes)                                         -> bench_{pesq,c3,c5,pesq_aligned*}.json
#   6. smoke()                                                          -> smoke.txt
# Every GPU step runs under its own time limit and the chain stops at the first failure.  The
# ISA statistics of the same build come from the CPU side (tools/isa_stats.py, see README).
# Usage: bash tools/closing_set.sh TAG [--no-tests]
set -o pipefail
R=$PWD
TAG=${1:?usage: closing_set.sh TAG [--no-tests]}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT $R/profiles/$TAG
if [ "${1:-}" != "--no-tests" ]; then
  bash tools/gpu_tests.sh $TAG || { echo "TESTS FAILED"; exit 1; }
fi
cd /tmp && export TMPDIR=/tmp
pmc() {  # pmc NAME COUNTERS...: one counter group, one run
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
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace_bench -o run --output-format csv -- python $R/bench.py --no-cpu-baseline > $OUT/bench_traced.json 2> $OUT/trace.log || { echo "TRACE FAILED"; tail -20 $OUT/trace.log; exit 1; }
cd $R
python tools/timeline.py $OUT/trace_bench > $OUT/timeline_bench.txt 2>&1 || exit 1
for w in pesq c3 c5 pesq_aligned pesq_aligned_utt pesq_aligned_p862; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "BENCH $w FAILED"; exit 1; }
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail $OUT/smoke.txt; exit 1; }
cat $OUT/smoke.txt
echo CLOSING_SET_DONE
