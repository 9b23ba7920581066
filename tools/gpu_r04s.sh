#!/bin/bash
# Round 4 iteration s: confidence with XCD bands by default (tests + timing vs the plain order),
# extraction with the block's tsdf staged in LDS (mode 11 vs 3), the integrate's XCD-grouped block
# order (variant 0x8000) against the default with the current kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_confidence.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r04s_tests.log 2>&1 || { tail -30 gpurun_out/r04s_tests.log; exit 1; }
tail -1 gpurun_out/r04s_tests.log
MQR_HIP_LIB="$PWD/tools/_ab/libmqr_ab.so" timeout -k 10 300 python -u tools/ab_extract.py --modes 3,11,19,27 --reps 21 > gpurun_out/r04s_ab1.json 2> gpurun_out/r04s_ab.err &&
MQR_HIP_LIB="$PWD/tools/_ab/libmqr_ab.so" timeout -k 10 300 python -u tools/ab_extract.py --modes 27,19,11,3 --reps 21 > gpurun_out/r04s_ab2.json 2>> gpurun_out/r04s_ab.err || { tail -20 gpurun_out/r04s_ab.err; exit 1; }
cat gpurun_out/r04s_ab1.json gpurun_out/r04s_ab2.json
MQR_HIP_LIB="$PWD/tools/_ab/libmqr_ab.so" timeout -k 10 400 python -u tools/ab_integrate.py --variants 0,0x8000 --rounds 5 --check > gpurun_out/r04s_int.json 2> gpurun_out/r04s_int.err || { tail -20 gpurun_out/r04s_int.err; exit 1; }
tail -5 gpurun_out/r04s_int.json
: > gpurun_out/r04s_conf.jsonl
for v in plain xcd xcd plain plain xcd; do
  MQR_HIP_LIB="$PWD/tools/_ab/libmqr_conf_$v.so" timeout -k 10 200 python -u tools/conf_workload.py --reps 7 > gpurun_out/r04s_tmp.json 2>> gpurun_out/r04s_conf.err || { tail -20 gpurun_out/r04s_conf.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r04s_tmp.json')); print(json.dumps({'lib': '$v', 'ms': d['ms_median'], 'digest': d['digest'], 'src': d['confidence_src']}))" >> gpurun_out/r04s_conf.jsonl
done
cat gpurun_out/r04s_conf.jsonl
