#!/bin/bash
# Bench A/B of the UNet snippet batch / VAE decode chunk sizes, alternating runs on one box.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "25 75" "30 90"; do
    set -- $cfg
    bash tools/hb.sh timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-validate \
      --snippet-batch $1 --vae-batch $2 > gpurun_out/batch_ab_$1_$2_$r.log 2>&1 || exit $?
    echo "sb=$1 vb=$2 run $r: $(grep '^{' gpurun_out/batch_ab_$1_$2_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["attention"]["frac"])')" >> gpurun_out/r04f_batch_ab.log
  done
done
