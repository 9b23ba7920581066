#!/bin/bash
# Round 4, first GPU call: the exchange tests (local twin at 2/3/8 ranks, one process per rank over
# gloo at 2/3/8), the confidence tests (NaN-distance fix), then a 2-rank rehearsal of the N>1 bench
# line (C4 split, gloo-staged merge: two ranks share the one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_confidence.py -m gpu -v --timeout 300 \
  --timeout-method thread > gpurun_out/r04a_tests.log 2>&1 || { tail -40 gpurun_out/r04a_tests.log; exit 1; }
tail -3 gpurun_out/r04a_tests.log
MQR_BENCH_WRAP_DEVICES=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 --weak-steps 5 \
  > gpurun_out/r04a_bench2.json 2> gpurun_out/r04a_bench2.err || { tail -30 gpurun_out/r04a_bench2.err; exit 1; }
tail -c 1500 gpurun_out/r04a_bench2.json
