#!/bin/bash
# Round-3 profiles: gather ceiling, rocprofv3 kernel stats of the bench, traffic passes, integrate /
# confidence / extraction counters, 4-byte-gather calibration of the fabric counters.  Each step
# under its own time limit; results under gpurun_out/ (profiles/ copies made by the scripts).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUND=${ROUND:-r03}
if [ -n "$TESTK" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "$TESTK" \
    > gpurun_out/iter_tests.log 2>&1 || { tail -30 gpurun_out/iter_tests.log; exit 1; }
  tail -2 gpurun_out/iter_tests.log
fi
timeout -k 10 120 tools/_ab/gather_ceiling > gpurun_out/gather_ceiling.jsonl || exit 1
cat gpurun_out/gather_ceiling.jsonl
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- \
  python3 bench.py --no-cpu --no-extras --no-c4 --no-c5 --steps 50 --warmup 5 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err \
  || { tail -20 gpurun_out/prof_bench.err; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
grep "mqr" gpurun_out/kernel_stats.csv | cut -c1-60,300-420 | head -12
echo "== traffic"
ROUND=$ROUND timeout -k 10 500 bash tools/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || { tail -20 gpurun_out/pmc_traffic.log; exit 1; }
mkdir -p gpurun_out/profiles_new && cp profiles/${ROUND}_pmc_traffic.json profiles/${ROUND}_pmc_fetch.csv profiles/${ROUND}_pmc_write.csv gpurun_out/profiles_new/
grep -E "traffic_over_alg|traffic_bytes_per_launch" profiles/${ROUND}_pmc_traffic.json | head -4
echo "== integrate counters"
KRE="k_integrate_lean" VARIANTS="0" timeout -k 10 500 bash tools/pmc_ab.sh > gpurun_out/pmc_ab_round.log 2>&1 || { tail -20 gpurun_out/pmc_ab_round.log; exit 1; }
cp gpurun_out/pmc_ab.json gpurun_out/profiles_new/${ROUND}_pmc_integrate_counters.json
echo "== confidence counters"
timeout -k 10 500 bash tools/pmc_conf.sh > gpurun_out/pmc_conf.log 2>&1 || { tail -5 gpurun_out/pmc_conf.log; exit 1; }
cp gpurun_out/pmc_conf.json gpurun_out/profiles_new/${ROUND}_pmc_confidence.json
grep -A8 '"derived"' gpurun_out/pmc_conf.json
echo "== extraction counters"
timeout -k 10 400 bash tools/pmc_kernels.sh 'k_mc_|k_pt_|k_scan|k_nb' --extract 3 > gpurun_out/pmck_extract.log 2>&1 || { tail -5 gpurun_out/pmck_extract.log; exit 1; }
echo "== calibration"
ROUND=$ROUND timeout -k 10 500 bash tools/pmc_calib.sh > gpurun_out/pmc_calib.log 2>&1 || { tail -5 gpurun_out/pmc_calib.log; exit 1; }
cp profiles/${ROUND}_pmc_calib.json gpurun_out/profiles_new/ 2>/dev/null
echo ALL_DONE
