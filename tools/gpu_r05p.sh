#!/bin/bash
# round 5 (p): config 3 occupancy A/B after the slope-form updates -- w6 (this build: 80
# VGPRs, 56 B of scratch whose stores reach HBM), w5 (96 VGPRs, no scratch), w4 (99)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
AB_ARGS="--config 3 --steps 10 --warmup 2" bash tools/ab.sh w6.so w5.so w4.so || exit $?
