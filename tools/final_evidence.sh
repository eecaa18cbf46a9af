#!/bin/bash
# Round-end evidence on one MI355X: GPU parity suite, smoke, every bench
# workload, and the rocprofv3 kernel trace + PMC passes of the default bench.
# Usage: tools/final_evidence.sh <tag>
TAG=${1:-r02f}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
timeout -k 10 200 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > gpurun_out/${TAG}_cfg3.json 2> gpurun_out/${TAG}_cfg3.err || exit 1
timeout -k 10 200 python bench.py --workload cfg4 --steps 50 > gpurun_out/${TAG}_cfg4.json 2> gpurun_out/${TAG}_cfg4.err || exit 1
timeout -k 10 200 python bench.py --workload cfg5 --steps 50 > gpurun_out/${TAG}_cfg5.json 2> gpurun_out/${TAG}_cfg5.err || exit 1
timeout -k 10 300 python bench.py --workload filesums > gpurun_out/${TAG}_filesums.json 2> gpurun_out/${TAG}_filesums.err || exit 1
bash tools/profile.sh $TAG
