#!/bin/bash
# GPU-box: bench workloads under two library builds (FSEM_LIB), alternating, two rounds.
# Usage: bash tools/ab_lib_bench.sh TAG LIB_A LIB_B WORKLOAD...
set -o pipefail
TAG=$1; A=$2; B=$3; shift 3
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
V=$PWD/fast_speech_enhancement_metrics_amd/lib/var
for r in 1 2; do
  for w in "$@"; do
    for L in $A $B; do
      FSEM_LIB=$V/$L.so timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > $OUT/${w}_${L}_$r.json 2> $OUT/${w}_${L}_$r.err || { echo "FAILED $w $L"; tail -5 $OUT/${w}_${L}_$r.err; exit 1; }
      python -c "import json,sys; d=json.load(open('$OUT/${w}_${L}_$r.json')); print('$w', '$L', $r, d['value'], d['ms_per_step'])"
    done
  done
done
