#!/bin/bash
# Round 4 iteration n: extraction A/B -- the emission grid over a compacted list of the blocks with
# output (mode bit 2) on top of modes 0 / 3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export MQR_HIP_LIB="$PWD/tools/_ab/libmqr_ab.so"
timeout -k 10 300 python -u tools/ab_extract.py --modes 3,7,0,4 --reps 21 > gpurun_out/r04n_ab1.json 2> gpurun_out/r04n_ab.err &&
timeout -k 10 300 python -u tools/ab_extract.py --modes 7,3,4,0,5,6 --reps 21 > gpurun_out/r04n_ab2.json 2>> gpurun_out/r04n_ab.err &&
cat gpurun_out/r04n_ab1.json gpurun_out/r04n_ab2.json
