#!/bin/bash
# round 5 (e): the tensor-schema ops + monomial adjoint on the GPU -- every GPU test, the
# config 5 bench twice (final_loss reproducible with the fixed ramp), its kernel stats and
# the config 5 PMC passes (adjoint + taped forward)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run() { local n=$1 secs=$2; shift 2; echo "== $n"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -2 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
run bench_c5a 300 python3 bench.py --config 5 --steps 100 --warmup 5 --no-cpu
run bench_c5b 300 python3 bench.py --config 5 --steps 100 --warmup 5 --no-cpu
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config 5 --no-cpu --steps 100 --warmup 5
bash tools/pmc_c5.sh
