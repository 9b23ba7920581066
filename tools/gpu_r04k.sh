#!/bin/bash
# Round 4 iteration k: the later batches' touches on a CU-masked stream (bit 25) at 32 / 64 / 128 CUs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_numerics.py -m gpu -q -k "specialised" --timeout 300 --timeout-method thread > gpurun_out/r04k_tests1.log 2>&1 \
  || { tail -40 gpurun_out/r04k_tests1.log; exit 1; }
tail -2 gpurun_out/r04k_tests1.log
for c in 32 64 128; do
  MQR_TOUCH_CUS=$c MQR_HIP_LIB=tools/_ab/libmqr_ab.so timeout -k 10 300 python tools/ab_integrate.py --variants 0,0x2000000 --rounds 7 --check \
    > gpurun_out/r04k_ab_$c.json 2> gpurun_out/r04k_ab.err || { tail -20 gpurun_out/r04k_ab.err; exit 1; }
  echo "cus=$c"; cat gpurun_out/r04k_ab_$c.json
done
