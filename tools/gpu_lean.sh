#!/bin/bash
# GPU check of the lean integrate kernels: numerics tests (exhaustive reciprocal checks, bit-equality
# of every variant), then an interleaved A/B of integrate variants on the bench workload.
# usage (on the box, via gpurun): bash tools/gpu_lean.sh "<variants>" [pytest -k expr]
set -o pipefail
V="${1:-0,40,41,42}"; K="${2:-}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_numerics.py -v --timeout 300 --timeout-method thread \
  ${K:+-k "$K"} > gpurun_out/num.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/num.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/ab_integrate.py --variants "$V" --rounds 4 > gpurun_out/ab.json 2> gpurun_out/ab.err
rc2=$?
cat gpurun_out/ab.json; tail -3 gpurun_out/ab.err
exit $rc2
