#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a ONE-GPU box: 2 ranks share cuda:0 over gloo
# (RCCL refuses two ranks on one device). Checks the launch contract (torchrun env,
# barrier + max-over-ranks timing, one JSON line from rank 0, config 4's gather), not
# scaling. Output under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local n=$1; shift; echo "== $n"; timeout -k 10 300 "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -2 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
for c in 2 4 5; do
  run rehearse_c$c python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29500 + c)) bench.py --gpus 2 --steps 5 \
    --warmup 2 --config $c --backend gloo
done
