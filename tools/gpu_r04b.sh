#!/bin/bash
# Round 4: full GPU suite, the default bench line, a rocprofv3 kernel-trace pass of the bench workload,
# the 2-rank rehearsal of the N>1 line (gloo-staged: both ranks on the one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1 \
  || { tail -40 gpurun_out/r04b_tests.log; exit 1; }
tail -2 gpurun_out/r04b_tests.log
timeout -k 10 500 python bench.py > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err || { tail -20 gpurun_out/r04b_bench.err; exit 1; }
python - <<'P'
import json; d=json.load(open("gpurun_out/r04b_bench.json"))
print({k: d[k] for k in ("value","ms_per_step","extract_ms")}, d["roofline"]["avg_launch_ms"], d["roofline"]["touch_ms_per_launch"], d["parity"]["all_ok"], d["c4"]["parity"]["all_ok"], d["c5"]["parity"]["all_ok"], d["confidence"]["ms"])
P
rm -rf gpurun_out/r04b_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04b_prof -o run -- \
  python bench.py --no-cpu --no-extras --steps 50 --warmup 5 > gpurun_out/r04b_prof_bench.json 2> gpurun_out/r04b_prof_bench.err \
  || { tail -20 gpurun_out/r04b_prof_bench.err; exit 1; }
find gpurun_out/r04b_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04b_kernel_stats.csv \;
find gpurun_out/r04b_prof -name "*kernel_trace.csv" -exec cp {} gpurun_out/r04b_kernel_trace.csv \;
grep "mqr" gpurun_out/r04b_kernel_stats.csv | cut -c1-60,300-420 | head -14
MQR_BENCH_WRAP_DEVICES=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 --weak-steps 5 \
  > gpurun_out/r04b_bench2.json 2> gpurun_out/r04b_bench2.err || { tail -30 gpurun_out/r04b_bench2.err; exit 1; }
python - <<'P'
import json; d=json.load(open("gpurun_out/r04b_bench2.json"))
print({k: d[k] for k in ("value","ms_per_step","merge_ms","merge_transport","scaling")}, d["parity"], d["weak_c2"])
P
MQR_HIP_LIB=tools/_ab/libmqr_ab.so timeout -k 10 300 python tools/ab_integrate.py --variants 0,23,24,25,26,0x20000 --rounds 7 --check \
  > gpurun_out/r04b_ab.json 2> gpurun_out/r04b_ab.err || { tail -20 gpurun_out/r04b_ab.err; exit 1; }
cat gpurun_out/r04b_ab.json
timeout -k 10 200 python tools/conf_workload.py --reps 5 --stats > gpurun_out/r04b_conf.json 2> gpurun_out/r04b_conf.err || { tail -20 gpurun_out/r04b_conf.err; exit 1; }
cat gpurun_out/r04b_conf.json
timeout -k 10 200 python tools/ab_extract.py --modes 0,1 --reps 15 > gpurun_out/r04b_abx.json 2> gpurun_out/r04b_abx.err || { tail -20 gpurun_out/r04b_abx.err; exit 1; }
cat gpurun_out/r04b_abx.json
