#!/bin/bash
# GPU-box: edge/stage parity tests, the whole GPU suite, then the bench (no CPU legs).
# Usage: bash tools/r3_check.sh TAG
set -o pipefail
TAG=${1:-r3}
OUT=$PWD/gpurun_out/$TAG; mkdir -p $OUT
bash tools/gpu_pytest.sh $TAG tests/test_edges_ref_gpu.py tests/test_stage_api_gpu.py > $OUT/edges_summary.txt 2>&1
echo "edges rc=$?"
grep -E "engine|passed|failed" $OUT/edges_summary.txt | grep -v "print(" | tail -40
bash tools/gpu_tests.sh ${TAG}_all > $OUT/all_summary.txt 2>&1
echo "all rc=$?"
tail -6 $OUT/all_summary.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
echo "bench rc=$?"
cat $OUT/bench.json
