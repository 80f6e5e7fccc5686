#!/bin/bash
# One GPU-box session: parity tests, smoke, bench (+ optional rocprof). Each GPU step has
# its own time limit; a crash / abort / timeout ends the session (test FAILURES do not).
# usage: bash tools/gpu_session.sh [tests|smoke|bench|prof|pmc]...
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abort session (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 900 python -m pytest tests -m gpu -q -x -rf ;;
    testsall) run pytest_gpu 900 python -m pytest tests -m gpu -q -rf ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    benchq) run bench 600 python bench.py --steps 20 --warmup 3 ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --steps 20 --warmup 3 ;;
    pmc) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
         run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2
         run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2
         run pmc_valu 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_valu -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2 ;;
    pmcflops) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
         run pmc_flops 600 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_flops -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2 ;;
    pmcstall) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
         run pmc_stall 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_stall -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2 ;;
    counters) run counters 120 rocprofv3 -L ;;
    pmcissue) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
         run pmc_issue 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_issue -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2 ;;
    ab) run ab 900 bash tools/ab.sh $(cd optiland_pr_amd/lib/variants && ls *.so) ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
