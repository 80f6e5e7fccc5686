#!/bin/bash
# round 5 (t): taped forward occupancy after the slope-form updates: fwd4 (this build, 128
# VGPRs), fwd3 (133, no scratch), fwd5 (96, 144 B of scratch) -- config 5 step
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
AB_ARGS="--config 5 --steps 200 --warmup 10" bash tools/ab.sh fwd4.so fwd3.so fwd5.so || exit $?
