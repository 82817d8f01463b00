#!/bin/bash
# DIAGNOSTIC: sustained FULL4 rates of the ablation builds named on the
# command line, then SQ counters of the first two.
set -o pipefail
bash tools/diag/gpu_sus_full4.sh "$@" || exit $?
bash tools/diag/gpu_sq_full4.sh "$1" "$2"
