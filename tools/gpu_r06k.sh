#!/bin/bash
# round 6 (k): the fast evaluations' steep-normal test as two magnitude compares and the
# (1 + k) r2 numerator test skipped when 1 + k == 1 -- A/B of config 3 against the committed
# kernels (variant prev), then the GPU suite (the fast pass must stay bit-identical).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -6 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
AB_ARGS="--config 3 --steps 10 --warmup 2" run r06k_ab_c3 900 bash tools/ab.sh prev.so ../liboptiland_rt.so
run r06k_pytest 900 python3 -u -m pytest --maxfail=10 -q --timeout 120 --timeout-method thread -m gpu tests/
echo END_OK
