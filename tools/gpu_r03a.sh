#!/bin/bash
# Round-3 validation + counter passes, in priority order; any failing step ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_iter.sh "$1" --no-c5 --no-c4 || exit 1
timeout -k 10 300 python3 -u tools/time_merge.py > gpurun_out/time_merge.json 2> gpurun_out/time_merge.err || { tail -5 gpurun_out/time_merge.err; exit 1; }
tail -1 gpurun_out/time_merge.json
MQR_HIP_LIB=$GRAFT_REPO_ROOT/tools/_ab/libmqr_ab.so timeout -k 10 300 python3 -u tools/ab_integrate.py --variants 0,6,7 --rounds 5 > gpurun_out/ab_pair.json 2> gpurun_out/ab_pair.err || { tail -5 gpurun_out/ab_pair.err; exit 1; }
cat gpurun_out/ab_pair.json | tail -5
timeout -k 10 400 bash tools/pmc_conf.sh > gpurun_out/pmc_conf.log 2>&1 || { tail -5 gpurun_out/pmc_conf.log; exit 1; }
timeout -k 10 400 bash tools/pmc_kernels.sh 'k_mc_|k_pt_|k_scan' --extract 3 > gpurun_out/pmck_extract.log 2>&1 || { tail -5 gpurun_out/pmck_extract.log; exit 1; }
timeout -k 10 500 bash tools/pmc_calib.sh > gpurun_out/pmc_calib.log 2>&1 || { tail -5 gpurun_out/pmc_calib.log; exit 1; }
echo ALL_DONE
