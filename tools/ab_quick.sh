#!/bin/bash
# GPU-box: in-process A/B of library variants -- the joint front end alone (tools/ab_front.py,
# bitwise check of the Bark bands / powers against the first variant) and the whole joint call
# (tools/ab_joint.py).  No GPU tests.  Usage: bash tools/ab_quick.sh TAG VAR...
set -o pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python tools/ab_front.py "$@" --rounds 8 > $OUT/ab_front.txt 2>&1 || { tail -5 $OUT/ab_front.txt; exit 1; }
cat $OUT/ab_front.txt | grep -v "^{"
timeout -k 10 300 python tools/ab_joint.py "$@" --rounds 8 > $OUT/ab_joint.txt 2>&1 || { tail -5 $OUT/ab_joint.txt; exit 1; }
grep median $OUT/ab_joint.txt
