#!/bin/bash
# round 6 (i): NURBS surfaces (ort_nurbs.h) -- GPU suite; A/B of config 3 with the fast asphere
# coordinate checks folded (coord_ok) against the committed kernels (variant head).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -6 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
AB_ARGS="--config 3 --steps 10 --warmup 2" run r06i_ab_c3 900 bash tools/ab.sh head.so ../liboptiland_rt.so
run r06i_pytest 900 python3 -u -m pytest --maxfail=10 -q --timeout 120 --timeout-method thread -m gpu tests/

echo END_OK
