#!/bin/bash
# scratch: attention shapes, twice
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/kbench.py --only attn || exit 1
timeout -k 10 200 python -u tools/kbench.py --only attn || exit 1
