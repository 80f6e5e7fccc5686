#!/bin/bash
# round 6 (h): fast-asphere quotients with the range test folded into one lens_range check and
# the Newton statistics by ballots -- GPU suite, then A/B of config 3 and config 2 against the
# committed kernels (variant head, build_variant.py --from-rev HEAD).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -6 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
run r06h_pytest 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
AB_ARGS="--config 3 --steps 10 --warmup 2" run r06h_ab_c3 900 bash tools/ab.sh head.so ../liboptiland_rt.so
AB_ARGS="--config 2 --steps 10 --warmup 2" run r06h_ab_c2 900 bash tools/ab.sh head.so ../liboptiland_rt.so
echo END_OK
