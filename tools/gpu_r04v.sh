#!/bin/bash
# Round 4 iteration v: confidence with the reference depth read and the outputs non-temporal (nt) vs
# the default (xcd), process-alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/r04v_conf.jsonl
for v in xcd nt nt xcd xcd nt nt xcd; do
  MQR_HIP_LIB="$PWD/tools/_ab/libmqr_conf_$v.so" timeout -k 10 200 python -u tools/conf_workload.py --reps 7 > gpurun_out/r04v_tmp.json 2>> gpurun_out/r04v_conf.err || { tail -20 gpurun_out/r04v_conf.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r04v_tmp.json')); print(json.dumps({'lib': '$v', 'ms': d['ms_median'], 'digest': d['digest'], 'src': d['confidence_src']}))" >> gpurun_out/r04v_conf.jsonl
done
cat gpurun_out/r04v_conf.jsonl
