#!/bin/bash
# GPU-box: A/B of stoi_tob's band sums (VALU segmented sums vs the MFMA contraction at 4 / 3
# waves per SIMD) inside the whole joint call, then the GPU tests on the default library.
# Usage: bash tools/r4_tob.sh TAG
set -o pipefail
TAG=${1:-tob}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u tools/ab_joint.py tob_valu tob_mfma4 tob_mfma3 --rounds 8 > $OUT/ab_joint.txt 2>&1 || { echo "AB FAILED"; tail -20 $OUT/ab_joint.txt; exit 1; }
tail -6 $OUT/ab_joint.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
