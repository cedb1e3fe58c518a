#!/bin/bash
# GPU-box quick check: parity tests, then the bench under a kernel trace (per-kernel times).
# Usage: bash tools/quick.sh TAG [bench args]
set -o pipefail
R=$PWD
TAG=${1:-q}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
bash tools/bench_trace.sh $TAG "$@" || exit 1
python tools/timeline.py $OUT/trace_bench | tail -8
