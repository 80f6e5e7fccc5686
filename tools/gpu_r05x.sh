#!/bin/bash
# round 5 (x): taped forward with the hybrid Zernike slopes (hyb) vs the reference's polar
# chain in the forward TU only (fchain): rocprofv3 kernel averages, alternating, one box
set -u
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
rm -f gpurun_out/ab.log
AB_ARGS="--config 5 --steps 200 --warmup 10" bash tools/ab_prof.sh "_kernel<" hyb.so fchain.so || exit $?
AB_ARGS="--config 5 --steps 200 --warmup 10" bash tools/ab_prof.sh "_kernel<" hyb.so fchain.so || exit $?
timeout -k 10 300 python3 bench.py --config 5 --steps 100 --warmup 5 > gpurun_out/bench_c5x.log 2>&1 || exit $?
