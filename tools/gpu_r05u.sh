#!/bin/bash
# round 5 (u): the final tree's GPU suite, smoke and bench lines (tools/gpu_r05_end.sh),
# then an A/B of the adjoint with its newest Newton iterate loaded with the surface's rows
# (tkpre, ORT_ADJ_TK_PREFETCH) against this build (base)
set -u
cd "$(dirname "$0")/.."
bash tools/gpu_r05_end.sh || exit $?
AB_ARGS="--config 5 --steps 200 --warmup 10" bash tools/ab.sh base.so tkpre.so || exit $?
