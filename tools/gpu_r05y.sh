#!/bin/bash
# round 5 (y): what the taped forward waits on -- base vs no tape rows 0-5 (notape),
# unconditional statistics atomics (atom), schedule read through a scalar load (ssched):
# rocprofv3 kernel averages of trace_kernel<5204u>, alternating, one box. The three
# variants were built from temporary -D switches in ort_kernels.h (tape rows 0-5 skipped;
# atomicAnd / atomicMax without the read; U = cst(a.sched)[readfirstlane(index)]),
# removed again after the measurement (profiles/r05_ab_fwd_waits.log)
set -u
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
rm -f gpurun_out/ab.log
for rep in 1 2; do
AB_ARGS="--config 5 --steps 200 --warmup 10" bash tools/ab_prof.sh "5204u" base.so notape.so atom.so ssched.so || exit $?
done
