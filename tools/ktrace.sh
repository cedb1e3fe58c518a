#!/bin/bash
# Kernel-trace summary of one_step.py (args passed through), e.g.  bash tools/ktrace.sh jt --joint
set -o pipefail
R=$PWD
TAG=${1:-kt}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python $R/tools/one_step.py --reps 3 "$@" > $OUT/trace.log 2>&1 || { echo "TRACE FAILED"; tail -20 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e6:8.3f} ms')
PY
