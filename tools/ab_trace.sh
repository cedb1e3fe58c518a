#!/bin/bash
# GPU-box: per-kernel A/B of library variants under a kernel trace.  Each round runs every
# variant (lib/var/NAME.so) as its own `one_step.py --joint` process under
# `rocprofv3 --kernel-trace`, in alternating order; tools/ab_trace_summary.py then reports the
# median duration of every engine kernel and of the joint step (first start to last end of a
# call) per variant.  Usage: bash tools/ab_trace.sh TAG ROUNDS VAR...
set -o pipefail
R=$PWD
TAG=$1; shift
ROUNDS=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for rd in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    export FSEM_LIB=$R/fast_speech_enhancement_metrics_amd/lib/var/$v.so
    timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/tr_${v}_$rd -o run --output-format csv -- python $R/tools/one_step.py --joint --reps 10 > $OUT/tr_${v}_$rd.log 2>&1 || { echo "TRACE $v FAILED"; tail -20 $OUT/tr_${v}_$rd.log; exit 1; }
  done
done
cd $R
python tools/ab_trace_summary.py $OUT "$@" | tee $OUT/ab_trace.txt
