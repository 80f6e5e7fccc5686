#!/bin/bash
# round 4 (r2): config 5 adjoint PMC passes (HBM bytes, fp64 FLOPs, VALU) with the final
# build, then the N=2 launch-contract rehearsal (gloo, two ranks on one GPU)
set -u
cd "$(dirname "$0")/.."
bash tools/pmc_c5.sh || exit $?
bash tools/rehearse_multirank.sh || exit $?
