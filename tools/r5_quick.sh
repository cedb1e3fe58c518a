#!/bin/bash
# GPU-box: selected GPU tests plus the drop-in fast-path A/B.  Usage: bash tools/r5_quick.sh TAG
set -o pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_dropin_fast_gpu.py tests/test_multidevice_gpu.py tests/test_bench_gpu.py tests/test_streams_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python tools/ab_dropin_fast.py > $OUT/ab_dropin_fast.txt 2>&1 || { tail -5 $OUT/ab_dropin_fast.txt; exit 1; }
cat $OUT/ab_dropin_fast.txt
if [ -n "${AB_VARIANTS:-}" ]; then bash tools/ab_quick.sh $TAG $AB_VARIANTS || exit 1; fi
