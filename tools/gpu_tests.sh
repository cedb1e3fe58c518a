#!/bin/bash
# GPU-box: the gpu test suite (one pytest process, per-test timeout).  Usage: bash tools/gpu_tests.sh TAG [pytest args]
set -o pipefail
OUT=$PWD/gpurun_out/${1:-gt}; shift; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" > $OUT/gpu_tests.log 2>&1
rc=$?
tail -25 $OUT/gpu_tests.log
exit $rc
