#!/bin/bash
# round 6 (g): the Newton statistics by ballots (main build) -- GPU suite, then A/B against
# the shuffle reductions (variant shfl, -DORT_SHFL_REPORT) on config 3 and config 5.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -6 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
run r06g_pytest 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
AB_ARGS="--config 3 --steps 10 --warmup 2" run r06g_ab_c3 900 bash tools/ab.sh shfl.so ../liboptiland_rt.so
AB_ARGS="--config 5 --steps 100 --warmup 5" run r06g_ab_c5 900 bash tools/ab.sh shfl.so ../liboptiland_rt.so
echo END_OK
