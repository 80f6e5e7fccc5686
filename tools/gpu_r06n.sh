#!/bin/bash
# round 6 (n): NURBS kernel throughput (tools/nurbs_rate.py).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python3 tools/nurbs_rate.py > gpurun_out/r06n_nurbs_rate.log 2>&1
rc=$?; tail -3 gpurun_out/r06n_nurbs_rate.log; exit $rc
