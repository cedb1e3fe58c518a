#!/bin/bash
# GPU-box: the joint engine on row chunks over two streams with the persistent front end's grid
# capped to fewer CUs (FSEM_FRONT_CUS), so the previous chunk's STOI tail and PESQ back end run on
# the CUs it leaves free (VERDICT r4 item 2's partitioned grid), against the serial plan.
# Usage: bash tools/probes/ab_partition.sh TAG CHUNK CHUNKS CAP...
set -o pipefail
TAG=$1; CHUNK=$2; CHUNKS=$3; shift 3
OUT=$PWD/gpurun_out/$TAG; mkdir -p $OUT
for cap in 0 "$@"; do
  FSEM_FRONT_CUS=$cap timeout -k 10 300 python tools/probes/ab_overlap.py --chunk $CHUNK --chunks $CHUNKS --rounds 6 > $OUT/cap_$cap.txt 2>&1 || { tail -5 $OUT/cap_$cap.txt; exit 1; }
  echo "cap $cap:"; grep -v amdgpu.ids $OUT/cap_$cap.txt
done
