#!/bin/bash
# HBM-traffic passes over one bench step (no warm-up, no validation, no CPU leg): FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 runs (TCC slots: 3 + 2 > 4), each under its own kill timeout.
#   PRESET=fast OUT=gpurun_out/pmc_bench bash tools/pmc_bench.sh
# then tools/bench_traffic.py turns the two CSVs into bench_traffic.json, and tools/traffic_split.py splits
# them per kernel and launch shape (each pass also writes the launch sequence, RDMI_PROF_SEQ → seq.json).
set -e
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/pmc_bench}
PRESET=${PRESET:-fast}
EXTRA=${EXTRA:-}
mkdir -p $OUT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  mkdir -p $OUT/$c
  RDMI_PROF_SEQ=$OUT/$c/seq.json timeout -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --pmc $c --output-format csv \
    -d $OUT/$c -o run -- python3 bench.py --preset $PRESET --steps 1 --warmup 0 --no-cpu-baseline --no-validate \
    $EXTRA > $OUT/$c.log 2>&1
  echo "$c ok"
done
