#!/bin/bash
# Round 4 iteration o: confidence decisions in boolean form + lerps along v first -- tests, then
# process-alternating timing of the old / new / new-with-SLP libraries (tools/build_conf_variants.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_confidence.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1 || { tail -30 gpurun_out/r04o_tests.log; exit 1; }
tail -1 gpurun_out/r04o_tests.log
: > gpurun_out/r04o_conf.jsonl
for v in old new slp slp new old old new slp; do
  MQR_HIP_LIB="$PWD/tools/_ab/libmqr_conf_$v.so" timeout -k 10 200 python -u tools/conf_workload.py --reps 7 > gpurun_out/r04o_tmp.json 2>> gpurun_out/r04o_conf.err || { tail -20 gpurun_out/r04o_conf.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r04o_tmp.json')); print(json.dumps({'lib': '$v', 'ms': d['ms_median'], 'digest': d['digest'], 'src': d['confidence_src']}))" >> gpurun_out/r04o_conf.jsonl
done
cat gpurun_out/r04o_conf.jsonl
