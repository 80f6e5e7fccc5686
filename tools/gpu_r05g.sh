#!/bin/bash
# round 5 (g): every GPU test (incl. the CUDA-key opcheck / torch.compile tests), then an
# A/B of config 3 (Horner even-asphere sums, unrolled) against the pre-Horner build, and
# config 5 on the current build
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--config 3 --steps 10 --warmup 2" bash tools/ab.sh main.so horner.so || exit $?
AB_ARGS="--config 5 --steps 100 --warmup 10" bash tools/ab.sh horner.so || exit $?
