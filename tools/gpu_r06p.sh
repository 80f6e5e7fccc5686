#!/bin/bash
# round 6 (p): the final build (NURBS solves inlined again) -- NURBS throughput, GPU suite,
# smoke, the default bench line and config 5.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -3 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
run r06p_nurbs_rate 300 python3 tools/nurbs_rate.py
run r06p_pytest 900 python3 -u -m pytest --maxfail=10 -q --timeout 120 --timeout-method thread -m gpu tests/
run r06p_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run r06p_bench 300 python3 bench.py
run r06p_bench_c5 400 python3 bench.py --config 5 --steps 100 --warmup 5 --no-cpu
echo END_OK
