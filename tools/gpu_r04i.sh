#!/bin/bash
# Round 4 iteration i: integrate stream-priority / head A/B (fixed priorities), 9 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_numerics.py -m gpu -q -k "specialised or exact_fallback" --timeout 300 --timeout-method thread > gpurun_out/r04i_tests1.log 2>&1 \
  || { tail -40 gpurun_out/r04i_tests1.log; exit 1; }
tail -2 gpurun_out/r04i_tests1.log
MQR_HIP_LIB=tools/_ab/libmqr_ab.so timeout -k 10 400 python tools/ab_integrate.py --variants 0,0x2000000,0x800000,0x2800000 --rounds 9 --check \
  > gpurun_out/r04i_ab.json 2> gpurun_out/r04i_ab.err || { tail -20 gpurun_out/r04i_ab.err; exit 1; }
cat gpurun_out/r04i_ab.json
