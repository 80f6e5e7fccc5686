#!/bin/bash
# round 6 (a): the GPU suite on the schedule-aware adjoint (standard / noll Zernike
# gradients, per-tensor fused Adam), the launch-floor experiment, then config 5 in both
# schemes with their kernel stats. Output: gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -4 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
run r06a_pytest 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
run r06a_launch_floor 120 tools/launch_floor/launch_floor
run r06a_c5_fringe 400 python3 bench.py --config 5 --steps 100 --warmup 5 --no-cpu
run r06a_c5_standard 400 python3 bench.py --config 5 --steps 100 --warmup 5 --no-cpu --zernike-scheme standard
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run r06a_prof_c5_standard 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06a_prof_c5s -o run -- python3 bench.py --config 5 --no-cpu --steps 50 --warmup 2 --zernike-scheme standard
run r06a_prof_c5_fringe 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06a_prof_c5f -o run -- python3 bench.py --config 5 --no-cpu --steps 50 --warmup 2
echo END_OK
