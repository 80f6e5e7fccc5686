#!/bin/bash
# round 6 (j): Newton statistics formed per evaluation by wave ballots (wstat) -- GPU suite
# (NURBS included), then A/B of config 3 and config 5 against the committed kernels
# (variant prev: ort_k_trace_mono.hip + ort_k_trace_tape.hip at HEAD).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -6 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
AB_ARGS="--config 3 --steps 10 --warmup 2" run r06j_ab_c3 900 bash tools/ab.sh prev.so ../liboptiland_rt.so
AB_ARGS="--config 5 --steps 100 --warmup 5" run r06j_ab_c5 900 bash tools/ab.sh prev.so ../liboptiland_rt.so
run r06j_pytest 900 python3 -u -m pytest --maxfail=10 -q --timeout 120 --timeout-method thread -m gpu tests/
echo END_OK
