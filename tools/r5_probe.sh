#!/bin/bash
# GPU-box probe (round 5): rocprofv3 counter list, then pesq_front phase stamps of variants.
# Usage: bash tools/r5_probe.sh TAG STAMP_VARIANT...
set -o pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "counter list failed (continuing: no GPU work ran)"
cd - >/dev/null
timeout -k 10 300 python tools/stamps_ab.py "$@" > $OUT/stamps_ab.txt 2>&1 || { tail -5 $OUT/stamps_ab.txt; exit 1; }
cat $OUT/stamps_ab.txt
# two-stream chunk overlap: front end at 2 (default) and 1 workgroup(s) per CU
timeout -k 10 300 python tools/ab_overlap.py --chunk 2048 --chunks 4 --rounds 6 > $OUT/overlap_2wg.txt 2>&1 || { tail -5 $OUT/overlap_2wg.txt; exit 1; }
cat $OUT/overlap_2wg.txt
FSEM_FRONT_WGS_PER_CU=1 timeout -k 10 300 python tools/ab_overlap.py --chunk 2048 --chunks 4 --rounds 6 > $OUT/overlap_1wg.txt 2>&1 || { tail -5 $OUT/overlap_1wg.txt; exit 1; }
cat $OUT/overlap_1wg.txt
FSEM_FRONT_WGS_PER_CU=1 timeout -k 10 300 python tools/ab_overlap.py --chunk 1024 --chunks 8 --rounds 6 > $OUT/overlap_1wg_1024.txt 2>&1 || { tail -5 $OUT/overlap_1wg_1024.txt; exit 1; }
cat $OUT/overlap_1wg_1024.txt
