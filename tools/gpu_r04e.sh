#!/bin/bash
# Round 4 iteration e: full GPU suite with the new defaults (full first batch, in-kernel exact path), the
# integrate A/B against the round-3 kernel / 64-frame head, per-kernel extraction times (rocprofv3), the
# confidence counters of the branch-free mode, confidence A/B, bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1 \
  || { tail -40 gpurun_out/r04e_tests.log; exit 1; }
tail -2 gpurun_out/r04e_tests.log
MQR_HIP_LIB=tools/_ab/libmqr_ab.so timeout -k 10 300 python tools/ab_integrate.py --variants 0,15,0x200000,0x100000 --rounds 7 --check \
  > gpurun_out/r04e_ab.json 2> gpurun_out/r04e_ab.err || { tail -20 gpurun_out/r04e_ab.err; exit 1; }
cat gpurun_out/r04e_ab.json
rm -rf /tmp/exprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/exprof -o run -- python tools/ab_extract.py --modes 0,1 --reps 15 \
  > gpurun_out/r04e_abx.json 2> gpurun_out/r04e_abx.err || { tail -20 gpurun_out/r04e_abx.err; exit 1; }
cat gpurun_out/r04e_abx.json
find /tmp/exprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04e_extract_kernel_stats.csv \;
grep -E "k_mc|k_pt" gpurun_out/r04e_extract_kernel_stats.csv | cut -c1-200 || true
MQR_CONF_MODE=3 timeout -k 10 400 bash tools/pmc_conf.sh > gpurun_out/r04e_pmc_conf.log 2>&1 || { tail -20 gpurun_out/r04e_pmc_conf.log; exit 1; }
cp gpurun_out/pmc_conf.json gpurun_out/r04e_pmc_conf_mode3.json
timeout -k 10 200 python tools/conf_workload.py --reps 5 --stats --ab 3 > gpurun_out/r04e_conf.json 2> gpurun_out/r04e_conf.err || { tail -20 gpurun_out/r04e_conf.err; exit 1; }
cat gpurun_out/r04e_conf.json
timeout -k 10 400 python bench.py > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err || { tail -20 gpurun_out/r04e_bench.err; exit 1; }
python - <<'P'
import json; d=json.load(open("gpurun_out/r04e_bench.json"))
print({k: d[k] for k in ("value","ms_per_step","extract_ms")}, d["roofline"]["avg_launch_ms"], d["parity"]["all_ok"], d["c4"]["parity"]["all_ok"], d["c5"]["parity"]["all_ok"], d["confidence"]["ms"])
P
