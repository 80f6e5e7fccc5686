#!/bin/bash
# round 6 (c): the GPU suite on the compact, fully written tape (opcheck on the taped
# path), the launch-floor chain experiment, smoke, config 2 and config 5 (both schemes),
# the A/B of the exact near-axis jet (variant no_disc). Output: gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -4 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
run r06c_pytest 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
run r06c_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run r06c_launch_floor 120 tools/launch_floor/launch_floor
run r06c_c2 300 python3 bench.py --steps 50 --warmup 5
run r06c_c5_fringe 400 python3 bench.py --config 5 --steps 100 --warmup 5 --no-cpu
run r06c_c5_standard 400 python3 bench.py --config 5 --steps 100 --warmup 5 --no-cpu --zernike-scheme standard
AB_ARGS="--config 5 --steps 100 --warmup 5" run r06c_ab_disc 900 bash tools/ab.sh no_disc.so ../liboptiland_rt.so
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run r06c_prof_floor 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06c_prof_floor -o run -- tools/launch_floor/launch_floor
run r06c_prof_c5_fringe 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06c_prof_c5f -o run -- python3 bench.py --config 5 --no-cpu --steps 50 --warmup 2
echo END_OK
