#!/bin/bash
# Round-3 evidence + A/B in one call: full GPU test suite (failures do not stop the call, a crash or
# timeout does), smoke, the default bench line, the integrate A/B (variants in $AB_VARIANTS), the
# merge timing tool.  Results under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations 15 \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests.log
grep -E "FAILED|ERROR" gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
if [ -n "$AB_VARIANTS" ]; then
  MQR_HIP_LIB=$GRAFT_REPO_ROOT/tools/_ab/libmqr_ab.so timeout -k 10 300 python3 -u tools/ab_integrate.py \
    --variants "$AB_VARIANTS" --rounds 5 --check > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  tail -12 gpurun_out/ab.json
fi
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -c 1200 gpurun_out/bench.json
echo
if [ -z "$NO_MERGE" ]; then
  timeout -k 10 300 python3 -u tools/time_merge.py > gpurun_out/time_merge.json 2> gpurun_out/time_merge.err || { tail -5 gpurun_out/time_merge.err; exit 1; }
  tail -c 600 gpurun_out/time_merge.json
fi
echo ALL_DONE
