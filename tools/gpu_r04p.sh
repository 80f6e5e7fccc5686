#!/bin/bash
# round 4 (p): A/B of non-temporal pupil loads (configs 2 and 4); config 2 PMC passes
# (HBM bytes with the non-temporal stores, fp64 FLOPs, VALU, stalls) + kernel statistics
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
rm -f gpurun_out/ab.log
AB_ARGS="--config 2 --steps 100 --warmup 10" bash tools/ab.sh base.so ntpupil.so || exit $?
AB_ARGS="--config 4 --steps 5 --warmup 2" bash tools/ab.sh base.so ntpupil.so || exit $?
bash tools/gpu_session.sh prof pmc pmcflops pmcstall || exit $?
