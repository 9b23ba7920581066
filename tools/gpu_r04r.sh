#!/bin/bash
# Round 4 iteration r: extraction A/B -- emission by a grid of at most 8 workgroups per CU walking the
# list of blocks with output (mode 7 = NIB + MAP + LST) against the default (3).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export MQR_HIP_LIB="$PWD/tools/_ab/libmqr_ab.so"
timeout -k 10 300 python -u tools/ab_extract.py --modes 3,7 --reps 21 > gpurun_out/r04r_ab1.json 2> gpurun_out/r04r_ab.err &&
timeout -k 10 300 python -u tools/ab_extract.py --modes 7,3 --reps 21 > gpurun_out/r04r_ab2.json 2>> gpurun_out/r04r_ab.err &&
cat gpurun_out/r04r_ab1.json gpurun_out/r04r_ab2.json
# confidence: XCD-banded tile order vs the default
: > gpurun_out/r04r_conf.jsonl
for v in new xcd xcd new new xcd xcd new new xcd xcd new; do
  MQR_HIP_LIB="$PWD/tools/_ab/libmqr_conf_$v.so" timeout -k 10 200 python -u tools/conf_workload.py --reps 7 > gpurun_out/r04r_tmp.json 2>> gpurun_out/r04r_conf.err || { tail -20 gpurun_out/r04r_conf.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r04r_tmp.json')); print(json.dumps({'lib': '$v', 'ms': d['ms_median'], 'digest': d['digest'], 'src': d['confidence_src']}))" >> gpurun_out/r04r_conf.jsonl
done
cat gpurun_out/r04r_conf.jsonl
