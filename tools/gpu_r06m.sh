#!/bin/bash
# round 6 (m): surface records loaded one surface ahead (variant pref, -DORT_PREFETCH_SURF)
# vs the final build -- config 5 (taped forward) and config 3, alternating on one box.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -6 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
AB_ARGS="--config 5 --steps 100 --warmup 5" run r06m_ab_c5 900 bash tools/ab.sh pref.so ../liboptiland_rt.so
AB_ARGS="--config 3 --steps 10 --warmup 2" run r06m_ab_c3 900 bash tools/ab.sh pref.so ../liboptiland_rt.so
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
ORT_LIB_PATH=optiland_pr_amd/lib/variants/pref.so run r06m_prof_pref 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06m_prof_pref -o run -- python3 bench.py --config 5 --no-cpu --steps 50 --warmup 5
run r06m_prof_main 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06m_prof_main -o run -- python3 bench.py --config 5 --no-cpu --steps 50 --warmup 5
echo END_OK
