#!/bin/bash
# round 6 (d): the marginal cost of a device-verified round in config 5's captured step
# (tools/rounds_probe.py) and the launch floor with a large kernel body. Output: gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -4 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
run r06d_launch_floor 120 tools/launch_floor/launch_floor
run r06d_rounds 600 python3 tools/rounds_probe.py
echo END_OK
