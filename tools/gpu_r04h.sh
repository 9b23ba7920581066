#!/bin/bash
# Round 4 iteration h: confidence neighbour loop A/B (default vs the ballot-gated deferral update of
# the A/B library), integrate stream-priority / head A/B, extraction counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_confidence.py tests/test_gpu_numerics.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04h_tests1.log 2>&1 \
  || { tail -40 gpurun_out/r04h_tests1.log; exit 1; }
tail -2 gpurun_out/r04h_tests1.log
for i in 1 2; do
  timeout -k 10 200 python tools/conf_workload.py --reps 7 > gpurun_out/r04h_conf_main$i.json 2> gpurun_out/r04h_conf.err || { tail -20 gpurun_out/r04h_conf.err; exit 1; }
  cat gpurun_out/r04h_conf_main$i.json
  MQR_HIP_LIB=tools/_ab/libmqr_ab.so timeout -k 10 200 python tools/conf_workload.py --reps 7 > gpurun_out/r04h_conf_ab$i.json 2> gpurun_out/r04h_conf.err || { tail -20 gpurun_out/r04h_conf.err; exit 1; }
  cat gpurun_out/r04h_conf_ab$i.json
done
MQR_HIP_LIB=tools/_ab/libmqr_ab.so timeout -k 10 300 python tools/ab_integrate.py --variants 0,0x2000000,0x800000,0x2800000 --rounds 7 --check \
  > gpurun_out/r04h_ab.json 2> gpurun_out/r04h_ab.err || { tail -20 gpurun_out/r04h_ab.err; exit 1; }
cat gpurun_out/r04h_ab.json
timeout -k 10 400 bash tools/pmc_extract.sh > gpurun_out/r04h_pmc_extract.log 2>&1 || { tail -20 gpurun_out/r04h_pmc_extract.log; exit 1; }
cat gpurun_out/r04h_pmc_extract.log
