#!/bin/bash
# round 5 (z): taped Zernike forward occupancy on the hybrid-slope build: 4 waves per SIMD
# (f4, 128 VGPRs, no scratch) vs 5 (f5, 96 VGPRs, 136 B): rocprofv3 kernel averages
set -u
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
rm -f gpurun_out/ab.log
for rep in 1 2; do
AB_ARGS="--config 5 --steps 200 --warmup 10" bash tools/ab_prof.sh "5204u" f4.so f5.so || exit $?
done
