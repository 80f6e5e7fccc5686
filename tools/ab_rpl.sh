#!/bin/bash
# A/B of rays-per-lane of the closed-form kernel (ORT_RPL)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in 1 2 4; do
    out=$(ORT_RPL=$v timeout -k 10 300 python bench.py --no-cpu --steps 200 --warmup 20 2>/dev/null | tail -1) || exit $?
    echo "rpl=$v rep$rep $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms']*1e3,2), 'us', '%.3e'%d['value'])")" | tee -a gpurun_out/ab.log
  done
done
