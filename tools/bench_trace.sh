#!/bin/bash
# rocprofv3 kernel trace + stats of the bench command itself (the roofline's kernel timing
# must agree with this summary).  Usage: bash tools/bench_trace.sh TAG [bench args]
set -o pipefail
R=$PWD
TAG=${1:-bt}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace_bench -o run --output-format csv -- python $R/bench.py --no-cpu-baseline "$@" > $OUT/bench_traced.json 2> $OUT/trace.log || { echo "TRACE FAILED"; tail -20 $OUT/trace.log; exit 1; }
cat $OUT/bench_traced.json
python3 - $OUT <<'PY'
import csv, glob, sys
out = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(out + "/trace_bench/**/*kernel_trace.csv", recursive=True)[0])))
front = [r for r in rows if "pesq_front" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in front]
print("pesq_front launches", len(d), "ms:", " ".join(f"{x:.3f}" for x in d))
PY
