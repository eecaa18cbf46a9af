#!/bin/bash
# Round-end evidence on one MI355X: GPU parity suite, smoke, every bench
# workload, and the rocprofv3 kernel trace + PMC passes of the cfg2 and cfg3
# benches (tools/gpu_run.sh steps).  Usage: tools/final_evidence.sh <tag>
bash tools/gpu_run.sh ${1:-r04z} tests smoke bench cfg3 cfg4 cfg5 filesums receive prof_cfg2 prof_cfg3
