#!/bin/bash
# Round 4 iteration j: extraction emission A/B -- the library (neighbour offsets read in the triangle
# pass) vs the A/B library (plus vertex / triangle waves split), alternating; extraction tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tsdf.py tests/test_gpu_merge.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04j_tests1.log 2>&1 \
  || { tail -40 gpurun_out/r04j_tests1.log; exit 1; }
tail -2 gpurun_out/r04j_tests1.log
for i in 1 2 3; do
  timeout -k 10 200 python tools/ab_extract.py --modes 0 --reps 21 > gpurun_out/r04j_abx_main$i.json 2> gpurun_out/r04j_abx.err || { tail -20 gpurun_out/r04j_abx.err; exit 1; }
  cat gpurun_out/r04j_abx_main$i.json
  MQR_HIP_LIB=tools/_ab/libmqr_ab.so timeout -k 10 200 python tools/ab_extract.py --modes 0 --reps 21 > gpurun_out/r04j_abx_ab$i.json 2> gpurun_out/r04j_abx.err || { tail -20 gpurun_out/r04j_abx.err; exit 1; }
  cat gpurun_out/r04j_abx_ab$i.json
done
