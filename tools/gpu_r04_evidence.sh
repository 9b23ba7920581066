#!/bin/bash
# Round-4 evidence in one call (run when the kernels are final): full GPU suite, smoke, the default
# bench line, a rocprofv3 --kernel-trace --stats pass of the bench workload, the FETCH / WRITE traffic
# passes, the integrate counters and the confidence counters -- each record tagged with the build
# (mqr_build_tag) so bench.py quotes it.  Summaries land in gpurun_out/profiles_new/ (copy into profiles/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/profiles_new
export TMPDIR=/tmp
ROUND=${ROUND:-r04}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/ev_tests.log 2>&1 \
    || { tail -40 gpurun_out/ev_tests.log; exit 1; }
  tail -2 gpurun_out/ev_tests.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev_smoke.log 2>&1 || { tail -20 gpurun_out/ev_smoke.log; exit 1; }
  tail -1 gpurun_out/ev_smoke.log
fi
ROUND=$ROUND bash tools/pmc_traffic.sh > gpurun_out/ev_pmc_traffic.log 2>&1 || { tail -20 gpurun_out/ev_pmc_traffic.log; exit 1; }
cp profiles/${ROUND}_pmc_traffic.json profiles/${ROUND}_pmc_fetch.csv profiles/${ROUND}_pmc_write.csv gpurun_out/profiles_new/
KRE="k_integrate_lean" VARIANTS="0" timeout -k 10 400 bash tools/pmc_ab.sh > gpurun_out/ev_pmc_ab.log 2>&1 || { tail -20 gpurun_out/ev_pmc_ab.log; exit 1; }
cp gpurun_out/pmc_ab.json gpurun_out/profiles_new/${ROUND}_pmc_integrate_counters.json
timeout -k 10 400 bash tools/pmc_conf.sh > gpurun_out/ev_pmc_conf.log 2>&1 || { tail -20 gpurun_out/ev_pmc_conf.log; exit 1; }
cp gpurun_out/pmc_conf.json gpurun_out/profiles_new/${ROUND}_pmc_confidence.json
cp gpurun_out/profiles_new/${ROUND}_pmc_*.json profiles/
timeout -k 10 200 python tools/conf_workload.py --reps 5 --stats --ab 4 > gpurun_out/profiles_new/${ROUND}_conf_workload.json 2> gpurun_out/ev_conf.err || { tail -20 gpurun_out/ev_conf.err; exit 1; }
cat gpurun_out/profiles_new/${ROUND}_conf_workload.json
timeout -k 10 200 python tools/ab_extract.py --modes 0 --reps 15 > gpurun_out/profiles_new/${ROUND}_extract_workload.json 2> gpurun_out/ev_abx.err || { tail -20 gpurun_out/ev_abx.err; exit 1; }
timeout -k 10 400 bash tools/pmc_extract.sh > gpurun_out/ev_pmc_extract.log 2>&1 || { tail -20 gpurun_out/ev_pmc_extract.log; exit 1; }
cp gpurun_out/pmc_extract.json gpurun_out/profiles_new/${ROUND}_pmc_extract.json
rm -rf /tmp/ev_exprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d /tmp/ev_exprof -o run -- \
  python tools/ab_extract.py --modes 0 --reps 15 > gpurun_out/ev_exprof.json 2> gpurun_out/ev_exprof.err \
  || { tail -20 gpurun_out/ev_exprof.err; exit 1; }
find /tmp/ev_exprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/profiles_new/${ROUND}_extract_kernel_stats.csv \;
timeout -k 10 500 python bench.py > gpurun_out/ev_bench.json 2> gpurun_out/ev_bench.err || { tail -20 gpurun_out/ev_bench.err; exit 1; }
cp gpurun_out/ev_bench.json gpurun_out/profiles_new/${ROUND}_bench.json
python - <<'P'
import json; d=json.load(open("gpurun_out/ev_bench.json"))
print({k: d[k] for k in ("value","ms_per_step","extract_ms")}, d["roofline"], d["parity"]["all_ok"], d["c4"]["parity"]["all_ok"], d["c5"]["parity"]["all_ok"], d["confidence"]["ms"], d["build"])
P
rm -rf /tmp/ev_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/ev_prof -o run -- \
  python bench.py --no-cpu --no-extras --steps 50 --warmup 5 > gpurun_out/ev_prof_bench.json 2> gpurun_out/ev_prof_bench.err \
  || { tail -20 gpurun_out/ev_prof_bench.err; exit 1; }
find /tmp/ev_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/profiles_new/${ROUND}_bench_kernel_stats.csv \;
grep "mqr" gpurun_out/profiles_new/${ROUND}_bench_kernel_stats.csv | cut -c1-60,300-420 | head -14
echo evidence done
