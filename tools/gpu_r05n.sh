#!/bin/bash
# round 5 (n): A/B in one box -- head (round-5 commit c6c7244), noslope (this tree's loop
# with the reference's normal-form update), slope (this tree): config 3 and config 5
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
AB_ARGS="--config 3 --steps 10 --warmup 2" bash tools/ab.sh head.so noslope.so slope.so || exit $?
AB_ARGS="--config 5 --steps 200 --warmup 10" bash tools/ab.sh head.so noslope.so slope.so || exit $?
