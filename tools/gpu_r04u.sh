#!/bin/bash
# Round 4 iteration u: XCD-banded pinhole ray casting -- ray-cast tests on the product library, then
# process-alternating timing of the plain / banded libraries (tools/build_ray_variants.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_raycast.py tests/test_gpu_color.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04u_tests.log 2>&1 || { tail -30 gpurun_out/r04u_tests.log; exit 1; }
tail -1 gpurun_out/r04u_tests.log
: > gpurun_out/r04u_ray.jsonl
for v in plain xcd xcd plain plain xcd xcd plain; do
  MQR_HIP_LIB="$PWD/tools/_ab/libmqr_ray_$v.so" timeout -k 10 200 python -u tools/raycast_workload.py --reps 7 >> gpurun_out/r04u_ray.jsonl 2>> gpurun_out/r04u_ray.err || { tail -20 gpurun_out/r04u_ray.err; exit 1; }
done
cat gpurun_out/r04u_ray.jsonl
