# Host-side A/B of a bench config: the committed tree copied to _ab_old/ against the
# working tree, interleaved on one box (host speed differs from box to box).
# AB_ARGS="--config 5 --steps 40 --warmup 5" bash tools/ab_host.sh
set -e
ARGS=${AB_ARGS:-"--config 5 --steps 40 --warmup 5"}
ms() { python3 -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])"; }
for i in 1 2 3; do
  echo "old $( (cd _ab_old && timeout -k 10 200 python bench.py $ARGS --no-cpu) | ms)"
  echo "new $(timeout -k 10 200 python bench.py $ARGS --no-cpu | ms)"
done
