#!/bin/bash
# Round 4 iteration p: confidence at 8 waves per SIMD (amdgpu_waves_per_eu) -- process-alternating
# timing of the variant libraries (tools/build_conf_variants.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/r04p_conf.jsonl
for v in new w8 slpw8 old old slpw8 w8 new new w8 slpw8 old; do
  MQR_HIP_LIB="$PWD/tools/_ab/libmqr_conf_$v.so" timeout -k 10 200 python -u tools/conf_workload.py --reps 7 > gpurun_out/r04p_tmp.json 2>> gpurun_out/r04p_conf.err || { tail -20 gpurun_out/r04p_conf.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r04p_tmp.json')); print(json.dumps({'lib': '$v', 'ms': d['ms_median'], 'digest': d['digest'], 'src': d['confidence_src']}))" >> gpurun_out/r04p_conf.jsonl
done
cat gpurun_out/r04p_conf.jsonl
