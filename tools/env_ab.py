"""Interleaved A/B of a launch-time switch (an RDMI_* variable the library reads per launch) on one of
tools/kbench.py's benchmarks, all variants in one process (guide §5.4 rule 24).

    python tools/env_ab.py --var RDMI_ATTN_SPREAD --values 0,1 --bench attn [--rounds 3] [--iters 10]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import kbench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--var", required=True)
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--bench", required=True, help="kbench function suffix: attn, conv, gnconv, gemm, ...")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    fn = getattr(kbench, "bench_" + a.bench)
    for r in range(a.rounds):
        for v in a.values.split(","):
            os.environ[a.var] = v
            print(f"== round {r} {a.var}={v}", flush=True)
            fn(a.iters)


if __name__ == "__main__":
    main()
