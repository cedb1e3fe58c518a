#!/bin/bash
# GPU-box probe: bench (no CPU baseline) then the pesq_front phase stamps (diagnostic build).
# Usage: bash tools/probe_stamps.sh TAG
set -o pipefail
R=$PWD
TAG=${1:-ps}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
FSEM_LIB=$R/fast_speech_enhancement_metrics_amd/lib/libfsem_stamps.so JOINT=1 timeout -k 10 300 python tools/stamps.py > $OUT/stamps.txt 2>&1 || { echo "STAMPS FAILED"; tail -20 $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
