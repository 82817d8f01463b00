#!/bin/bash
# DIAGNOSTIC: one 20-ply launch's host round trip and event span with each
# kind of timing event (tools/diag/single_launch.py, $NARDE_EVENTS), twice.
set -o pipefail
cd "$(dirname "$0")/../.."
for rep in 1 2; do
  for k in torch nofence default todevice; do
    NARDE_EVENTS=$k timeout -k 5 90 python tools/diag/single_launch.py ref2 1 20 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
