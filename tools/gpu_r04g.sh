#!/bin/bash
# Round 4 iteration g: the confidence and extraction GPU tests, confidence digest + timing (default
# branch-free lean stages vs the branchy mode 4) and stage counts, extraction per-kernel times with the
# wave-parallel look-back, the confidence counters, then the full suite and the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_confidence.py tests/test_gpu_tsdf.py tests/test_gpu_numerics.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04g_tests1.log 2>&1 \
  || { tail -40 gpurun_out/r04g_tests1.log; exit 1; }
tail -2 gpurun_out/r04g_tests1.log
timeout -k 10 200 python tools/conf_workload.py --reps 5 --stats --ab 4 > gpurun_out/r04g_conf.json 2> gpurun_out/r04g_conf.err || { tail -20 gpurun_out/r04g_conf.err; exit 1; }
cat gpurun_out/r04g_conf.json
rm -rf /tmp/exprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/exprof -o run -- python tools/ab_extract.py --modes 0 --reps 15 \
  > gpurun_out/r04g_abx.json 2> gpurun_out/r04g_abx.err || { tail -20 gpurun_out/r04g_abx.err; exit 1; }
cat gpurun_out/r04g_abx.json
find /tmp/exprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04g_extract_kernel_stats.csv \;
timeout -k 10 400 bash tools/pmc_conf.sh > gpurun_out/r04g_pmc_conf.log 2>&1 || { tail -20 gpurun_out/r04g_pmc_conf.log; exit 1; }
cp gpurun_out/pmc_conf.json gpurun_out/r04g_pmc_conf.json
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1 \
  || { tail -40 gpurun_out/r04g_tests.log; exit 1; }
tail -2 gpurun_out/r04g_tests.log
timeout -k 10 400 python bench.py > gpurun_out/r04g_bench.json 2> gpurun_out/r04g_bench.err || { tail -20 gpurun_out/r04g_bench.err; exit 1; }
python - <<'P'
import json; d=json.load(open("gpurun_out/r04g_bench.json"))
print({k: d[k] for k in ("value","ms_per_step","extract_ms")}, d["roofline"]["avg_launch_ms"], d["parity"]["all_ok"], d["c4"]["parity"]["all_ok"], d["c5"]["parity"]["all_ok"], d["confidence"]["ms"], d["c5"]["extract_ms"])
P
