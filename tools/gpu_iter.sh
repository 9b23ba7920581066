#!/bin/bash
# One GPU iteration: selected GPU tests, the bench line, a rocprofv3 kernel-trace pass of the bench.
# Usage (on the box, via gpurun): bash tools/gpu_iter.sh "<pytest -k expr or empty>" [bench args...]
set -o pipefail
K="$1"; shift
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" \
    > gpurun_out/iter_tests.log 2>&1 || { tail -30 gpurun_out/iter_tests.log; exit 1; }
  tail -2 gpurun_out/iter_tests.log
fi
timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err \
  || { tail -20 gpurun_out/iter_bench.err; exit 1; }
export TMPDIR=/tmp
rm -rf gpurun_out/iter_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/iter_prof -o run -- \
  python bench.py --no-cpu --no-extras --steps 3 --warmup 1 "$@" > gpurun_out/iter_prof.json 2> gpurun_out/iter_prof.err \
  || { tail -20 gpurun_out/iter_prof.err; exit 1; }
find gpurun_out/iter_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/iter_kernel_stats.csv \;
grep mqr gpurun_out/iter_kernel_stats.csv | cut -c1-50,200-400 | sed 's/(.*)"//' | head -20
