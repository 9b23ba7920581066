#!/bin/bash
# Round 4 iteration m: extraction A/B -- per-cube triangle counts from the count pass (mode 1),
# LDS row maps instead of the binary searches (mode 2), both (mode 3).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export MQR_HIP_LIB="$PWD/tools/_ab/libmqr_ab.so"
timeout -k 10 300 python -u tools/ab_extract.py --modes 0,1,2,3 --reps 21 > gpurun_out/r04m_ab1.json 2> gpurun_out/r04m_ab.err &&
timeout -k 10 300 python -u tools/ab_extract.py --modes 3,2,1,0 --reps 21 > gpurun_out/r04m_ab2.json 2>> gpurun_out/r04m_ab.err &&
cat gpurun_out/r04m_ab1.json gpurun_out/r04m_ab2.json
