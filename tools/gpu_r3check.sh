#!/bin/bash
# Bench sanity on the final tree: the default line and a short cfg3 line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py > gpurun_out/chk_bench.json 2> gpurun_out/chk_bench.err || exit 1
timeout -k 10 200 python bench.py --workload cfg3 --steps 2 --no-cpu > gpurun_out/chk_cfg3.json 2> gpurun_out/chk_cfg3.err || exit 2
