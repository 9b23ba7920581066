#!/bin/bash
# Round 4 iteration x: extraction with the triangles' neighbour row records prefetched during the
# vertex loop (mode 7) vs the default (3).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export MQR_HIP_LIB="$PWD/tools/_ab/libmqr_ab.so"
timeout -k 10 300 python -u tools/ab_extract.py --modes 3,7 --reps 21 > gpurun_out/r04x_ab1.json 2> gpurun_out/r04x_ab.err &&
timeout -k 10 300 python -u tools/ab_extract.py --modes 7,3 --reps 21 > gpurun_out/r04x_ab2.json 2>> gpurun_out/r04x_ab.err &&
cat gpurun_out/r04x_ab1.json gpurun_out/r04x_ab2.json
