#!/bin/bash
# GPU-box: the GPU tests on the in-tree library, then an in-process joint-call A/B of library
# variants (tools/ab_joint.py) and config-3 bench lines per variant.  Usage: bash tools/ab_round.sh TAG VAR...
set -o pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG; mkdir -p $OUT
bash tools/gpu_tests.sh $TAG || exit 1
timeout -k 10 300 python tools/ab_joint.py "$@" --rounds 10 > $OUT/ab_joint.txt 2>&1 || { tail -5 $OUT/ab_joint.txt; exit 1; }
grep median $OUT/ab_joint.txt
for v in "$@"; do
  FSEM_LIB=$PWD/fast_speech_enhancement_metrics_amd/lib/var/$v.so timeout -k 10 200 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c3_$v.json 2>/dev/null || exit 1
  echo c3 $v $(python -c "import json;d=json.load(open('$OUT/c3_$v.json'));print(d['ms_per_step'])")
done
