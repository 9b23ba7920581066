#!/bin/bash
# Round-3 validation + counter passes, in priority order; any failing step ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_iter.sh "$1" --no-c5 --no-c4 || exit 1
timeout -k 10 400 bash tools/pmc_conf.sh > gpurun_out/pmc_conf.log 2>&1 || { tail -5 gpurun_out/pmc_conf.log; exit 1; }
timeout -k 10 400 bash tools/pmc_kernels.sh 'k_mc_|k_pt_|k_scan' --extract 3 > gpurun_out/pmck_extract.log 2>&1 || { tail -5 gpurun_out/pmck_extract.log; exit 1; }
timeout -k 10 500 bash tools/pmc_calib.sh > gpurun_out/pmc_calib.log 2>&1 || { tail -5 gpurun_out/pmc_calib.log; exit 1; }
echo ALL_DONE
