#!/bin/bash
# round 5 end (2 of 2): the PMC passes behind the bench lines' traffic / FP64 figures --
# config 2 (kernel stats + HBM + compute), config 3 (compute, HBM), config 4 (HBM),
# config 5 (the adjoint and the taped forward). Output under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
bash tools/profile_round.sh || exit $?
bash tools/pmc_c3.sh || exit $?
bash tools/pmc_configs.sh || exit $?
bash tools/pmc_c5.sh || exit $?
echo PMC_OK
