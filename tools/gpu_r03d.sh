#!/bin/bash
# Round-3 evidence for the shipped default: full GPU suite, smoke, bench line, rocprofv3 kernel stats
# of the bench workload, FETCH / WRITE traffic passes of the integrate kernel.  Results under
# gpurun_out/ (profiles/ copies by the traffic script).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUND=${ROUND:-r03}
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations 15 \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests.log
grep -E "FAILED|ERROR" gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -c 400 gpurun_out/bench.json
echo
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- \
  python3 bench.py --no-cpu --no-extras --no-c4 --no-c5 --steps 50 --warmup 5 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err \
  || { tail -20 gpurun_out/prof_bench.err; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
grep "mqr" gpurun_out/kernel_stats.csv | cut -c1-60,300-420 | head -12
ROUND=$ROUND timeout -k 10 500 bash tools/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || { tail -20 gpurun_out/pmc_traffic.log; exit 1; }
mkdir -p gpurun_out/profiles_new && cp profiles/${ROUND}_pmc_traffic.json profiles/${ROUND}_pmc_fetch.csv profiles/${ROUND}_pmc_write.csv gpurun_out/profiles_new/
grep -E "traffic_over_alg|traffic_bytes_per_launch|\"kernel\"" profiles/${ROUND}_pmc_traffic.json | head -4
if [ -n "$WITH_COUNTERS" ]; then
  KRE="k_integrate_lean" VARIANTS="0" timeout -k 10 500 bash tools/pmc_ab.sh > gpurun_out/pmc_ab_round.log 2>&1 || { tail -20 gpurun_out/pmc_ab_round.log; exit 1; }
  cp gpurun_out/pmc_ab.json gpurun_out/profiles_new/${ROUND}_pmc_integrate_counters.json
fi
echo ALL_DONE
