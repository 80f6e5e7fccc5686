#!/bin/bash
# Secondary bench lines (BASELINE configs 1-5) + their rocprofv3 kernel stats.
# usage: bash tools/bench_configs.sh [prof]   (GPU box; output under gpurun_out/)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() { local n=$1 secs=$2; shift 2; echo "== $n: $*"; timeout -k 10 "$secs" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -3 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
run bench_c1 300 python3 bench.py --config 1 --steps 200 --warmup 5
run bench_c2 300 python3 bench.py --config 2 --steps 50 --warmup 5
run bench_c3 400 python3 bench.py --config 3 --steps 10 --warmup 2
run bench_c4 400 python3 bench.py --config 4 --steps 10 --warmup 2
run bench_c5 400 python3 bench.py --config 5 --steps 100 --warmup 5
if [ "${1:-}" = prof ]; then
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  for c in 1 3 4 5; do
    run prof_c$c 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c$c -o run -- python3 bench.py --config $c --no-cpu --steps 5 --warmup 1
  done
fi
