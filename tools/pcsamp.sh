#!/bin/bash
# PC sampling (rocprofv3 host-trap, beta) of one bench config: where the waves' time goes,
# per instruction. usage: bash tools/pcsamp.sh CONFIG [extra bench args]
# Afterwards on the build host: python tools/pcsamp_summary.py gpurun_out/pcs_cCONFIG
set -u
cd "$(dirname "$0")/.."
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out
c=$1; shift
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
  --pc-sampling-unit time --pc-sampling-interval 1 --output-format csv \
  -d gpurun_out/pcs_c$c -o run -- python3 bench.py --no-cpu --config $c --steps 20 --warmup 2 \
  --ramp-steps 0 "$@" > gpurun_out/pcs_c$c.log 2>&1
rc=$?; tail -3 gpurun_out/pcs_c$c.log; exit $rc
