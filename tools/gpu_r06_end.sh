#!/bin/bash
# round 6 end: the GPU suite, smoke(), the default bench line (config 2) under rocprofv3,
# bench lines of configs 1-5 (+ config 5 with the standard Zernike scheme) with their
# kernel stats. Output under gpurun_out/ (copied into profiles/r06_end_* afterwards).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -3 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
run r06e_pytest 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/
run r06e_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run r06e_bench 300 python3 bench.py
bash tools/bench_configs.sh prof || exit $?
run r06e_c5_standard 400 python3 bench.py --config 5 --steps 100 --warmup 5 --zernike-scheme standard
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run r06e_prof_c2 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06e_prof_c2 -o run -- python3 bench.py --no-cpu --steps 50 --warmup 5
cd "$(dirname "$0")/.." 2>/dev/null || true
AB_ARGS="--config 3 --steps 10 --warmup 2" run r06e_ab_slopemax 900 bash tools/ab.sh slopemax.so ../liboptiland_rt.so
echo END_OK
