#!/bin/bash
# Round 4 iteration q: the block-count scan without the list's third scan (template) -- extraction
# tests, extraction timing (A/B library: mode 0 vs the default 3) and the extraction kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tsdf.py -x -q --timeout 300 --timeout-method thread -k "mesh or points or extraction" > gpurun_out/r04q_tests.log 2>&1 || { tail -30 gpurun_out/r04q_tests.log; exit 1; }
tail -1 gpurun_out/r04q_tests.log
MQR_HIP_LIB="$PWD/tools/_ab/libmqr_ab.so" timeout -k 10 300 python -u tools/ab_extract.py --modes 3,0 --reps 21 > gpurun_out/r04q_ab1.json 2> gpurun_out/r04q_ab.err &&
MQR_HIP_LIB="$PWD/tools/_ab/libmqr_ab.so" timeout -k 10 300 python -u tools/ab_extract.py --modes 0,3 --reps 21 > gpurun_out/r04q_ab2.json 2>> gpurun_out/r04q_ab.err &&
timeout -k 10 200 python -u tools/ab_extract.py --modes 0 --reps 21 > gpurun_out/r04q_product.json 2>> gpurun_out/r04q_ab.err || { tail -20 gpurun_out/r04q_ab.err; exit 1; }
rm -rf /tmp/q_exprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d /tmp/q_exprof -o run -- \
  python tools/ab_extract.py --modes 0 --reps 15 > gpurun_out/r04q_exprof.json 2> gpurun_out/r04q_exprof.err \
  || { tail -20 gpurun_out/r04q_exprof.err; exit 1; }
find /tmp/q_exprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04q_extract_kernel_stats.csv \;
cat gpurun_out/r04q_ab1.json gpurun_out/r04q_ab2.json gpurun_out/r04q_product.json
grep "mqr" gpurun_out/r04q_extract_kernel_stats.csv | cut -c1-40,200-330
# confidence: the working-tree kernel at 7 vs 8 waves per SIMD, 8 alternations
: > gpurun_out/r04q_conf.jsonl
for v in new w8 w8 new new w8 w8 new new w8 w8 new new w8 w8 new; do
  MQR_HIP_LIB="$PWD/tools/_ab/libmqr_conf_$v.so" timeout -k 10 200 python -u tools/conf_workload.py --reps 7 > gpurun_out/r04q_tmp.json 2>> gpurun_out/r04q_conf.err || { tail -20 gpurun_out/r04q_conf.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r04q_tmp.json')); print(json.dumps({'lib': '$v', 'ms': d['ms_median'], 'digest': d['digest'], 'src': d['confidence_src']}))" >> gpurun_out/r04q_conf.jsonl
done
cat gpurun_out/r04q_conf.jsonl
