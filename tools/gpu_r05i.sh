#!/bin/bash
# round 5 (i): the rms spot size fused into the taped forward (F_RMS + ort_rms_finish, the
# gradient folded into the adjoint) and the fused Adam + patch: their GPU tests, then
# config 5 fused / unfused (ORT_FUSED_RMS=0) / torch Adam, kernel stats of the default
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_autograd.py tests/test_gpu_optim.py tests/test_gpu_graph_step.py tests/test_gpu_opcheck.py tests/test_gpu_adjoint.py > gpurun_out/pytest_i.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_i.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in fused unfused torchadam; do
    extra=""; envs=""
    [ $v = unfused ] && envs="ORT_FUSED_RMS=0"
    [ $v = torchadam ] && extra="--torch-adam"
    env $envs timeout -k 10 300 python3 bench.py --no-cpu --config 5 --steps 100 --warmup 10 $extra > gpurun_out/c5_$v.json 2> gpurun_out/c5_$v.err
    rc=$?; echo "$v rep$rep $(tail -c 600 gpurun_out/c5_$v.json)" >> gpurun_out/ab_i.log
    [ $rc -eq 0 ] || exit $rc
  done
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5i -o run -- python3 bench.py --config 5 --no-cpu --steps 100 --warmup 5 > gpurun_out/prof_c5i.log 2>&1
