#!/bin/bash
# Round 4 iteration t: with the XCD-banded order, the SLP-vectorised confidence (fewer VALU, 6 waves)
# against the default (7 waves without SLP... held to 8 in its production instances).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/r04t_conf.jsonl
for v in new slp slp new new slp slp new; do
  MQR_HIP_LIB="$PWD/tools/_ab/libmqr_conf_$v.so" timeout -k 10 200 python -u tools/conf_workload.py --reps 7 > gpurun_out/r04t_tmp.json 2>> gpurun_out/r04t_conf.err || { tail -20 gpurun_out/r04t_conf.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r04t_tmp.json')); print(json.dumps({'lib': '$v', 'ms': d['ms_median'], 'digest': d['digest'], 'src': d['confidence_src']}))" >> gpurun_out/r04t_conf.jsonl
done
cat gpurun_out/r04t_conf.jsonl
