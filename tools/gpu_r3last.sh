#!/bin/bash
# Final check of the committed tree: the whole GPU suite, smoke, default bench.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03x}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 200 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
