#!/bin/bash
# Round 4 iteration w: the emission pass's per-block work distribution on the C2 mesh.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/extract_block_hist.py > gpurun_out/r04w_hist.json 2> gpurun_out/r04w_hist.err || { tail -20 gpurun_out/r04w_hist.err; exit 1; }
cat gpurun_out/r04w_hist.json
