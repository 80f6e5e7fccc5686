#!/bin/bash
# round 6 (f): what config 3's deferred range checks cost (timing-only variant
# ORT_FAST_NOCHECK of the Newton kernels' TU), two alternating repetitions.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -6 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
AB_ARGS="--config 3 --steps 10 --warmup 2" run r06f_ab_c3_nochk 900 bash tools/ab.sh c3_nochk.so ../liboptiland_rt.so
echo END_OK
