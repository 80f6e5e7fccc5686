#!/bin/bash
# round 6 (q): rocprofv3 kernel statistics of the shipped build -- the NURBS lens
# (tools/nurbs_rate.py) and config 3.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
R=$PWD
cd /tmp && export TMPDIR=/tmp
prof() { local n=$1; shift; echo "== $n"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$n -o $n -- "$@" > $R/gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; grep '^{' $R/gpurun_out/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
prof r06q_nurbs python3 $R/tools/nurbs_rate.py
prof r06q_c3 python3 $R/bench.py --config 3 --steps 20 --warmup 3 --no-cpu
echo END_OK
