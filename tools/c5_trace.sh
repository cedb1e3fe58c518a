#!/bin/bash
# Kernel-trace summary of the config-5 bench workload.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${1:-c5}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python $R/bench.py --workload c5 --steps 2 --warmup 1 > $OUT/bench.json 2> $OUT/trace.log || { echo "TRACE FAILED"; tail -20 $OUT/trace.log; exit 1; }
cat $OUT/bench.json
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e6:8.3f} ms  total {float(r["TotalDurationNs"])/1e6:8.2f}')
PY
