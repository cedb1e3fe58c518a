#!/bin/bash
# One SQ counter pass over one_step.py (args passed through) -> per-kernel summary.
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${1:-pq}; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY -d $OUT/pmc_sq -o run --output-format csv -- python $R/tools/one_step.py --reps 1 "$@" > $OUT/pmc.log 2>&1 || { echo "PMC FAILED"; tail -20 $OUT/pmc.log; exit 1; }
python3 $R/tools/pmc_summary.py $OUT | python3 -c "
import json,sys
d=json.load(sys.stdin)
for k,v in d.items():
    wc=v.get('SQ_WAVE_CYCLES',1); w=max(1,v.get('SQ_WAVES',1))
    print(f\"{k[:40]:40s} waves {w:8.0f} cyc/wave {wc/w:9.0f} valu/wave {v.get('SQ_INSTS_VALU',0)/w:8.0f} lds/wave {v.get('SQ_INSTS_LDS',0)/w:7.0f} actVALU {v.get('SQ_ACTIVE_INST_VALU',0)/wc:5.2f} waitinst {v.get('SQ_WAIT_INST_ANY',0)/wc:5.2f} waitany {v.get('SQ_WAIT_ANY',0)/wc:5.2f} conf/lds {v.get('SQ_LDS_BANK_CONFLICT',0)/max(1,v.get('SQ_INSTS_LDS',1)):6.2f}\")
"
