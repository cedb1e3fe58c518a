#!/bin/bash
# GPU-box: per-row edge parity figures, the bench (with the CPU baseline) and the bench under a
# kernel trace (per-kernel times; the step timeline).  Usage: bash tools/r4_measure.sh TAG
set -o pipefail
TAG=${1:-m}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_edges_ref_gpu.py -s -q --timeout 120 --timeout-method thread > $OUT/edges_rows.log 2>&1 || { echo "EDGE TESTS FAILED"; tail -20 $OUT/edges_rows.log; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/bench_trace.sh $TAG > /dev/null || { echo "TRACE FAILED"; exit 1; }
python tools/timeline.py $OUT/trace_bench > $OUT/timeline_bench.txt 2>&1 || exit 1
tail -8 $OUT/timeline_bench.txt
