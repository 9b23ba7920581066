#!/bin/bash
# Round GPU evidence in one call: full GPU test suite, smoke, the default bench line (CPU baseline
# and parity included), a rocprofv3 --kernel-trace --stats pass of the bench workload, the
# FETCH/WRITE traffic passes and the integrate kernel's SQ/TA counters.  Everything lands in
# gpurun_out/ (copy the summaries into profiles/).  ROUND names the profile files (default r02).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUND=${ROUND:-r02}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -c 600 gpurun_out/bench.json
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- \
  python bench.py --no-cpu --no-extras --steps 50 --warmup 5 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err \
  || { tail -20 gpurun_out/prof_bench.err; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
grep "mqr" gpurun_out/kernel_stats.csv | cut -c1-60,300-420 | head -12
ROUND=$ROUND bash tools/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || { tail -20 gpurun_out/pmc_traffic.log; exit 1; }
grep -E "traffic_bytes_per_launch|alg_bytes_per_launch|traffic_over_alg|\"kernel\"" profiles/${ROUND}_pmc_traffic.json
mkdir -p gpurun_out/profiles_new && cp profiles/${ROUND}_pmc_traffic.json profiles/${ROUND}_pmc_fetch.csv profiles/${ROUND}_pmc_write.csv gpurun_out/profiles_new/
KRE="k_integrate_(lean|lt)" VARIANTS="0 3 5" timeout -k 10 700 bash tools/pmc_ab.sh > gpurun_out/pmc_ab_round.log 2>&1 || { tail -20 gpurun_out/pmc_ab_round.log; exit 1; }
cp gpurun_out/pmc_ab.json gpurun_out/profiles_new/${ROUND}_pmc_integrate_counters.json
echo round evidence done
