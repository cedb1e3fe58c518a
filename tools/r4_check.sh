#!/bin/bash
# GPU-box: an interleaved A/B of library variants (lib/var/*.so), the GPU tests and the tob
# diagnostic dump.  Usage: bash tools/r4_check.sh TAG VARIANT...
set -o pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
if [ $# -gt 0 ]; then
  timeout -k 10 400 python tools/ab_joint.py "$@" --rounds 10 > $OUT/ab_joint.txt 2>&1 || { echo "AB FAILED"; tail -5 $OUT/ab_joint.txt; exit 1; }
  grep -v amdgpu.ids $OUT/ab_joint.txt | tail -6
fi
bash tools/gpu_tests.sh $TAG || { echo "TESTS FAILED"; exit 1; }
timeout -k 10 120 python tools/tob_dump.py $OUT/tob_dump.npz tone_probe_10k edges_16k:dc1000_both lowpass_10k > $OUT/tob_dump.log 2>&1 || { echo "TOB DUMP FAILED"; exit 1; }
