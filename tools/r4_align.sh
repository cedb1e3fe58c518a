#!/bin/bash
# GPU-box: the time-alignment tests (row and utterance modes) and both aligned-PESQ bench lines.
# Usage: bash tools/r4_align.sh TAG
set -o pipefail
TAG=${1:-al}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_align_gpu.py tests/test_align_utt_gpu.py -v -s --timeout 200 --timeout-method thread > $OUT/align_tests.log 2>&1 || { echo "ALIGN TESTS FAILED"; tail -40 $OUT/align_tests.log; exit 1; }
tail -12 $OUT/align_tests.log
timeout -k 10 300 python bench.py --workload pesq_aligned_utt --no-cpu-baseline > $OUT/bench_pesq_aligned_utt.json 2> $OUT/bench_utt.err || { echo "BENCH UTT FAILED"; tail -20 $OUT/bench_utt.err; exit 1; }
cat $OUT/bench_pesq_aligned_utt.json
timeout -k 10 300 python bench.py --workload pesq_aligned --no-cpu-baseline > $OUT/bench_pesq_aligned.json 2> $OUT/bench_al.err || { echo "BENCH ROW FAILED"; tail -20 $OUT/bench_al.err; exit 1; }
cat $OUT/bench_pesq_aligned.json
