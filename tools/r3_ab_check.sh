#!/bin/bash
# GPU-box: kernel-trace A/B of variant libraries (VARS), then tools/r3_check.sh TAG.
set -o pipefail
TAG=${1:-r3}
VARS=${VARS:-"va vd"} bash tools/ab_trace.sh || exit 1
bash tools/r3_check.sh $TAG
