#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the config 3 and 4 trace
# kernels; then on the build host:
#   python tools/profile_hbm.py r02_config3 - gpurun_out/pmc_c3_* --traffic hbm_traffic_c3.json
set -u
cd "$(dirname "$0")/.."
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out
run() { local n=$1; shift; echo "== $n"; timeout -k 10 300 "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for c in 3 4; do
  B="python3 bench.py --no-cpu --config $c --steps 3 --warmup 1"
  run pmc_c${c}_fetch rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_c${c}_fetch -o run -- $B
  run pmc_c${c}_write rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_c${c}_write -o run -- $B
done
