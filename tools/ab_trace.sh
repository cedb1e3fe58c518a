#!/bin/bash
# Kernel-trace stats of one_step.py (ARGS, default --joint) for each variant library in lib/var (VARS="va vb")
set -o pipefail
R=$PWD
cd /tmp && export TMPDIR=/tmp
for v in ${VARS:-va vb}; do
OUT=$R/gpurun_out/abt_$v
FSEM_LIB=$R/fast_speech_enhancement_metrics_amd/lib/var/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python $R/tools/one_step.py --reps ${REPS:-8} ${ARGS---joint} > $OUT.log 2>&1 || { echo "TRACE FAILED $v"; tail -20 $OUT.log; exit 1; }
python3 - $OUT $v <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0])))
print(sys.argv[2], "  ".join(f'{r["Name"].split("(")[0].replace("void ","").replace("fsem::","")}={float(r["AverageNs"])/1e6:.3f}' for r in rows if "fsem" in r["Name"]))
PY
done
