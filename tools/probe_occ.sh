#!/bin/bash
# pesq_front time at 1 and 2 resident workgroups per CU (occupancy sensitivity).
set -o pipefail
OUT=$PWD/gpurun_out/${1:-occ}; mkdir -p $OUT
for w in 2 1; do
  FSEM_FRONT_WGS_PER_CU=$w timeout -k 10 200 python tools/time_kernels.py --reps 5 > $OUT/wg$w.txt 2>&1 || { tail $OUT/wg$w.txt; exit 1; }
  echo "wgs/cu=$w: $(tail -1 $OUT/wg$w.txt)"
done
