#!/bin/bash
# Round 4 iteration: numerics (variant equality incl. the touch variants), tsdf / mesh / points tests,
# the A/B library's variant equality, then integrate A/B (in-kernel exact path, two-phase touch) and the
# extraction time.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 \
  --timeout-method thread > gpurun_out/r04d_tests.log 2>&1 || { tail -40 gpurun_out/r04d_tests.log; exit 1; }
tail -2 gpurun_out/r04d_tests.log
MQR_HIP_LIB=tools/_ab/libmqr_ab.so timeout -k 10 300 python tools/ab_integrate.py --variants 0,0x100000,0x200000,0x400000,0x800000,23,24,0x80000,0x1000000 --rounds 7 --check \
  > gpurun_out/r04d_ab.json 2> gpurun_out/r04d_ab.err || { tail -20 gpurun_out/r04d_ab.err; exit 1; }
cat gpurun_out/r04d_ab.json
timeout -k 10 200 python tools/ab_extract.py --modes 0,1 --reps 15 > gpurun_out/r04d_abx.json 2> gpurun_out/r04d_abx.err || { tail -20 gpurun_out/r04d_abx.err; exit 1; }
cat gpurun_out/r04d_abx.json
timeout -k 10 200 python tools/conf_workload.py --reps 5 --diag --ab 3 > gpurun_out/r04d_conf.json 2> gpurun_out/r04d_conf.err || { tail -20 gpurun_out/r04d_conf.err; exit 1; }
cat gpurun_out/r04d_conf.json
timeout -k 10 300 python bench.py > gpurun_out/r04d_bench.json 2> gpurun_out/r04d_bench.err || { tail -20 gpurun_out/r04d_bench.err; exit 1; }
cat gpurun_out/r04d_bench.json
