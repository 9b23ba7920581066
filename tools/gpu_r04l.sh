#!/bin/bash
# Round 4 iteration l: confidence tests and timing (scalar-offset tap row, narrow deferral masks).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_confidence.py tests/test_gpu_distributed.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04l_tests1.log 2>&1 \
  || { tail -40 gpurun_out/r04l_tests1.log; exit 1; }
tail -2 gpurun_out/r04l_tests1.log
for i in 1 2; do
  timeout -k 10 200 python tools/conf_workload.py --reps 7 --stats > gpurun_out/r04l_conf$i.json 2> gpurun_out/r04l_conf.err || { tail -20 gpurun_out/r04l_conf.err; exit 1; }
  cat gpurun_out/r04l_conf$i.json
done
