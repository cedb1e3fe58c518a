#!/bin/bash
# GPU-box: one round's committed profile set -- parity tests, bench (with CPU baseline), the
# bench under a kernel trace (its pesq_front average must agree with the bench's event timing),
# the one-step joint trace and PMC passes (HBM bytes, SQ counters, LDS / VALU activity), and the
# config-2 (PESQ alone) / config-3 / config-5 bench lines.  Usage: bash tools/profile_round.sh TAG
set -o pipefail
R=$PWD
TAG=${1:-pr}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
bash tools/gpu_round.sh $TAG || exit 1
bash tools/bench_trace.sh $TAG || exit 1
python tools/timeline.py $OUT/trace_bench > $OUT/timeline_bench.txt 2>&1 || exit 1
bash tools/pmc_lds.sh $TAG --joint > $OUT/pmc_lds_valu.txt || exit 1
timeout -k 10 300 python bench.py --workload pesq --no-cpu-baseline > $OUT/bench_pesq.json 2> $OUT/bench_pesq.err || exit 1
timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 1
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 1
PMC_ROWS=4096 python tools/pmc_summary.py $OUT > $OUT/pmc_summary.json || exit 1
echo PROFILE_DONE
