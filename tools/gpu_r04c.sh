#!/bin/bash
# Round 4 iteration: confidence / tsdf tests, confidence timing + stage counts, the bench line, a
# kernel-trace pass (output kept in /tmp; stats + step head into gpurun_out), integrate A/B of the
# speculative head and the touch kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_confidence.py tests/test_gpu_tsdf.py tests/test_gpu_confidence_driver.py -m gpu -q --timeout 300 \
  --timeout-method thread > gpurun_out/r04c_tests.log 2>&1 || { tail -40 gpurun_out/r04c_tests.log; exit 1; }
tail -2 gpurun_out/r04c_tests.log
timeout -k 10 200 python tools/conf_workload.py --reps 5 --stats > gpurun_out/r04c_conf.json 2> gpurun_out/r04c_conf.err || { tail -20 gpurun_out/r04c_conf.err; exit 1; }
cat gpurun_out/r04c_conf.json
timeout -k 10 400 python bench.py --no-c5 --e2e-frames 0 > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err || { tail -20 gpurun_out/r04c_bench.err; exit 1; }
python - <<'P'
import json; d=json.load(open("gpurun_out/r04c_bench.json"))
print({k: d[k] for k in ("value","ms_per_step","extract_ms")}, d["roofline"]["avg_launch_ms"], d["roofline"]["touch_ms_per_launch"], d["parity"]["all_ok"], d["c4"]["parity"]["all_ok"], d["confidence"]["ms"])
P
rm -rf /tmp/r04c_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/r04c_prof -o run -- \
  python bench.py --no-cpu --no-extras --steps 50 --warmup 5 > gpurun_out/r04c_prof_bench.json 2> gpurun_out/r04c_prof_bench.err \
  || { tail -20 gpurun_out/r04c_prof_bench.err; exit 1; }
find /tmp/r04c_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04c_kernel_stats.csv \;
python3 tools/step_head.py $(find /tmp/r04c_prof -name "*kernel_trace.csv" | head -1) > gpurun_out/r04c_step_head.json
cat gpurun_out/r04c_step_head.json
MQR_HIP_LIB=tools/_ab/libmqr_ab.so timeout -k 10 300 python tools/ab_integrate.py --variants 0,0x40000,0x20000 --rounds 7 --check \
  > gpurun_out/r04c_ab.json 2> gpurun_out/r04c_ab.err || { tail -20 gpurun_out/r04c_ab.err; exit 1; }
cat gpurun_out/r04c_ab.json
