#!/bin/bash
# GPU-box: run the given test files in one pytest process with per-test timeouts, log to
# gpurun_out/TAG/t.log and print the result lines.  Usage: bash tools/gpu_pytest.sh TAG tests...
set -o pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest "$@" -v -s --timeout 300 --timeout-method thread > $OUT/t.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|engine|frames|sym|passed|failed" $OUT/t.log | tail -120
exit $rc
