#!/bin/bash
# One parameterised GPU call (replaces round 4's per-iteration tools/gpu_r04*.sh scripts).
#   STEPS="tests bench n2 ..." bash tools/gpu_step.sh      (run under gpurun, from the repo root)
# Steps, run in the order given, each under its own time limit, the call ending at the first failure:
#   tests       the whole `pytest -m gpu` suite                      -> gpurun_out/${TAG}_gpu_tests.log
#   tests:F     pytest -m gpu on the test files F (comma separated)   -> gpurun_out/${TAG}_gpu_tests.log
#   smoke       __graft_entry__.smoke()                               -> gpurun_out/${TAG}_smoke.log
#   bench       the default bench line (N = 1)                        -> gpurun_out/${TAG}_bench.json
#   benchq      a short bench (no C4 / C5 / drop-in legs)             -> gpurun_out/${TAG}_benchq.json
#   c5          the C5 leg alone, parity included (bench.py --c5-only)   -> gpurun_out/${TAG}_c5.json
#   n2          2-rank rehearsal on one GPU (gloo-staged merge)        -> gpurun_out/${TAG}_bench_n2.json
#   n2self      the same, bench.py --gpus 2 starting its own ranks (no torchrun) -> gpurun_out/${TAG}_bench_n2_selflaunch.json
#   mbytes      C4 exchange bytes / zero-weight voxels / per-rank times at 2, 4, 8 ranks (tools/merge_bytes.py)
#   steptrace   kernel trace of the C2 loop: step head (tools/step_head.py) and integrate-stream gaps (tools/integrate_gaps.py)
#   prof        rocprofv3 --kernel-trace --stats of the C2 bench      -> gpurun_out/${TAG}_bench_kernel_stats.csv
#   shardtrace[:W:R] one C4 shard's reset + integrate passes under a kernel trace (tools/shard_steps.py + step_head.py)
#   mprof       rocprofv3 kernel trace + stats of tools/time_merge.py (8 ranks on one GPU)
#   profc5      the same over the C5 leg alone                        -> gpurun_out/${TAG}_c5_kernel_stats.csv
#   xtrace      kernel trace of 30 extractions: wall vs device span vs gaps -> gpurun_out/${TAG}_extract_timeline.json
#   traffic     FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.sh) -> profiles/${TAG}_pmc_traffic.json
#   pmcint      SQ / TA / TCP counters of the default integrate kernel (tools/pmc_ab.sh) -> profiles_new/
#   pmcconf     counter passes of the confidence kernel (tools/pmc_conf.sh) -> profiles_new/${TAG}_pmc_confidence.json
#   abint:V     tools/ab_integrate.py over integrate variants V (comma separated, A/B library)
#   abext:M     tools/ab_extract.py over extraction modes M (A/B library)
#   d2h         device -> host copy ceilings (tools/d2h_probe.py) with 1 / 4 / 8 staging threads
#   chunkab     drop-in integrate() with 64- vs 127-frame hand-offs (tools/dropin_ab.py)
#   conf        tools/conf_workload.py (the confidence kernel alone)
#   abasync[:V] integrate_frames returning with its last integrate queued vs draining, or variants V (tools/ab_async.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
for step in ${STEPS:-tests}; do
  echo "== $step ($(date +%H:%M:%S))"
  case "$step" in
    tests)
      timeout -k 10 900 $PYT tests > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
      tail -1 gpurun_out/${TAG}_gpu_tests.log ;;
    tests:*)
      files=$(echo "${step#tests:}" | tr ',' ' ')
      timeout -k 10 900 $PYT $files > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
      tail -1 gpurun_out/${TAG}_gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
      tail -1 gpurun_out/${TAG}_smoke.log ;;
    bench)
      timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
      tail -c 400 gpurun_out/${TAG}_bench.json ;;
    benchq)
      timeout -k 10 600 python bench.py --no-c4 --no-c5 --e2e-frames 0 > gpurun_out/${TAG}_benchq.json 2> gpurun_out/${TAG}_benchq.err || { tail -30 gpurun_out/${TAG}_benchq.err; exit 1; }
      tail -c 400 gpurun_out/${TAG}_benchq.json ;;
    c5)
      timeout -k 10 900 python bench.py --c5-only > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || { tail -30 gpurun_out/${TAG}_c5.err; exit 1; }
      tail -c 1500 gpurun_out/${TAG}_c5.json ;;
    n2)
      MQR_BENCH_WRAP_DEVICES=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --weak-steps 10 \
        > gpurun_out/${TAG}_bench_n2.json 2> gpurun_out/${TAG}_bench_n2.err || { tail -40 gpurun_out/${TAG}_bench_n2.err; exit 1; }
      tail -c 600 gpurun_out/${TAG}_bench_n2.json ;;
    n2self)
      MQR_BENCH_WRAP_DEVICES=1 timeout -k 10 900 python bench.py --gpus 2 --steps 10 --warmup 2 --weak-steps 10 \
        > gpurun_out/${TAG}_bench_n2_selflaunch.json 2> gpurun_out/${TAG}_bench_n2_selflaunch.err || { tail -40 gpurun_out/${TAG}_bench_n2_selflaunch.err; exit 1; }
      tail -c 600 gpurun_out/${TAG}_bench_n2_selflaunch.json ;;
    mbytes)
      timeout -k 10 600 python tools/merge_bytes.py > gpurun_out/${TAG}_merge_bytes.json 2> gpurun_out/${TAG}_merge_bytes.err || { tail -30 gpurun_out/${TAG}_merge_bytes.err; exit 1; }
      tail -8 gpurun_out/${TAG}_merge_bytes.err ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- \
        python bench.py --no-cpu --no-extras --steps 50 --warmup 5 --touch-steps 0 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof_bench.err \
        || { tail -20 gpurun_out/${TAG}_prof_bench.err; exit 1; }
      find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_bench_kernel_stats.csv \;
      rm -rf gpurun_out/prof  # (traces: gpurun copies back at most 64 MiB of gpurun_out/)
      grep "mqr" gpurun_out/${TAG}_bench_kernel_stats.csv | cut -c1-70 | head -12 ;;
    steptrace)
      rm -rf gpurun_out/st
      timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d gpurun_out/st -o run -- \
        python bench.py --no-cpu --no-extras --no-c4 --no-c5 --e2e-frames 0 --steps 50 --warmup 5 --touch-steps 0 \
        > gpurun_out/${TAG}_st_bench.json 2> gpurun_out/${TAG}_st_bench.err || { tail -20 gpurun_out/${TAG}_st_bench.err; exit 1; }
      cp "$(find gpurun_out/st -name '*kernel_trace.csv' | head -1)" gpurun_out/${TAG}_step_trace.csv
      rm -rf gpurun_out/st
      python tools/step_head.py gpurun_out/${TAG}_step_trace.csv --steps 40 > gpurun_out/${TAG}_step_head.json && cat gpurun_out/${TAG}_step_head.json
      python tools/integrate_gaps.py gpurun_out/${TAG}_step_trace.csv > gpurun_out/${TAG}_integrate_gaps.json && cat gpurun_out/${TAG}_integrate_gaps.json ;;
    mprof)
      rm -rf gpurun_out/mp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/mp -o run -- \
        python tools/time_merge.py --ranks 8 --reps 5 > gpurun_out/${TAG}_time_merge.json 2> gpurun_out/${TAG}_time_merge.err \
        || { tail -20 gpurun_out/${TAG}_time_merge.err; exit 1; }
      find gpurun_out/mp -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_merge_kernel_stats.csv \;
      python tools/merge_trace.py "$(find gpurun_out/mp -name '*kernel_trace.csv' | head -1)" > gpurun_out/${TAG}_merge_timeline.json
      rm -rf gpurun_out/mp
      cat gpurun_out/${TAG}_time_merge.json; head -c 3000 gpurun_out/${TAG}_merge_timeline.json ;;
    shardtrace|shardtrace:*)
      WR=8:3; [ "$step" != shardtrace ] && WR="${step#shardtrace:}"
      rm -rf gpurun_out/sh
      timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/sh -o run -- \
        python tools/shard_steps.py --world "${WR%%:*}" --rank "${WR##*:}" --steps 40 > gpurun_out/${TAG}_shard_steps.json 2> gpurun_out/${TAG}_shard_steps.err \
        || { tail -20 gpurun_out/${TAG}_shard_steps.err; exit 1; }
      python tools/step_head.py "$(find gpurun_out/sh -name '*kernel_trace.csv' | head -1)" --steps 30 > gpurun_out/${TAG}_shard_head.json
      rm -rf gpurun_out/sh
      cat gpurun_out/${TAG}_shard_steps.json gpurun_out/${TAG}_shard_head.json ;;
    shardmerge)
      timeout -k 10 300 python tools/shard_steps.py --merge --steps 30 > gpurun_out/${TAG}_shard_merge.json 2> gpurun_out/${TAG}_shard_merge.err || { tail -20 gpurun_out/${TAG}_shard_merge.err; exit 1; }
      cat gpurun_out/${TAG}_shard_merge.json ;;
    shardall)
      timeout -k 10 300 python tools/shard_steps.py --all --steps 40 > gpurun_out/${TAG}_shard_all.json 2> gpurun_out/${TAG}_shard_all.err || { tail -20 gpurun_out/${TAG}_shard_all.err; exit 1; }
      grep "W=" gpurun_out/${TAG}_shard_all.err ;;
    profc5)
      rm -rf gpurun_out/profc5
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/profc5 -o run -- \
        python bench.py --c5-only --no-parity > gpurun_out/${TAG}_prof_c5.json 2> gpurun_out/${TAG}_prof_c5.err \
        || { tail -20 gpurun_out/${TAG}_prof_c5.err; exit 1; }
      find gpurun_out/profc5 -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_c5_kernel_stats.csv \;
      rm -rf gpurun_out/profc5
      grep "mqr" gpurun_out/${TAG}_c5_kernel_stats.csv | cut -c1-70 | head -16 ;;
    xtrace)
      rm -rf gpurun_out/xt
      timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/xt -o run -- \
        python tools/extract_timeline.py --run --walls gpurun_out/xt_walls.json > gpurun_out/${TAG}_xt.log 2>&1 || { tail -20 gpurun_out/${TAG}_xt.log; exit 1; }
      python tools/extract_timeline.py --analyze "$(find gpurun_out/xt -name '*kernel_trace.csv' | head -1)" gpurun_out/xt_walls.json \
        > gpurun_out/${TAG}_extract_timeline.json && cat gpurun_out/${TAG}_extract_timeline.json
      rm -rf gpurun_out/xt ;;
    traffic)
      ROUND=$TAG timeout -k 10 600 bash tools/pmc_traffic.sh > gpurun_out/${TAG}_pmc_traffic.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_traffic.log; exit 1; }
      mkdir -p gpurun_out/profiles_new && cp profiles/${TAG}_pmc_traffic.json profiles/${TAG}_pmc_fetch.csv profiles/${TAG}_pmc_write.csv gpurun_out/profiles_new/
      grep -E "traffic_bytes_per_launch|traffic_over_alg" profiles/${TAG}_pmc_traffic.json ;;
    pmcint)
      VARIANTS="0" timeout -k 10 700 bash tools/pmc_ab.sh > gpurun_out/${TAG}_pmc_ab.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_ab.log; exit 1; }
      mkdir -p gpurun_out/profiles_new && cp gpurun_out/pmc_ab.json gpurun_out/profiles_new/${TAG}_pmc_integrate_counters.json
      rm -rf /tmp/pmcab
      head -c 600 gpurun_out/pmc_ab.json ;;
    pmcconf)
      timeout -k 10 600 bash tools/pmc_conf.sh > gpurun_out/${TAG}_pmc_conf.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_conf.log; exit 1; }
      mkdir -p gpurun_out/profiles_new && cp gpurun_out/pmc_conf.json gpurun_out/profiles_new/${TAG}_pmc_confidence.json
      rm -rf /tmp/pmcconf
      head -c 400 gpurun_out/pmc_conf.json ;;
    abint:*)
      MQR_HIP_LIB="$PWD/tools/_ab/libmqr_ab.so" timeout -k 10 600 python -u tools/ab_integrate.py --check --rounds 7 --variants "${step#abint:}" \
        > gpurun_out/${TAG}_abint.json 2> gpurun_out/${TAG}_abint.err || { tail -20 gpurun_out/${TAG}_abint.err; exit 1; }
      cat gpurun_out/${TAG}_abint.json ;;
    abext:*)
      MQR_HIP_LIB="$PWD/tools/_ab/libmqr_ab.so" timeout -k 10 600 python -u tools/ab_extract.py --modes "${step#abext:}" --reps 21 \
        > gpurun_out/${TAG}_abext.json 2> gpurun_out/${TAG}_abext.err || { tail -20 gpurun_out/${TAG}_abext.err; exit 1; }
      cat gpurun_out/${TAG}_abext.json ;;
    d2h)
      for t in 1 4 8; do
        MQR_D2H_THREADS=$t timeout -k 10 120 python -u tools/d2h_probe.py >> gpurun_out/${TAG}_d2h.jsonl 2> gpurun_out/${TAG}_d2h.err || { tail -20 gpurun_out/${TAG}_d2h.err; exit 1; }
      done
      cat gpurun_out/${TAG}_d2h.jsonl ;;
    chunkab)
      timeout -k 10 600 python -u tools/dropin_ab.py > gpurun_out/${TAG}_chunk_ab.json 2> gpurun_out/${TAG}_chunk_ab.err || { tail -20 gpurun_out/${TAG}_chunk_ab.err; exit 1; }
      cat gpurun_out/${TAG}_chunk_ab.json ;;
    chunkprof)
      timeout -k 10 600 python -u tools/dropin_ab.py --profile --rounds 1 > gpurun_out/${TAG}_chunk_prof.json 2> gpurun_out/${TAG}_chunk_prof.txt || { tail -20 gpurun_out/${TAG}_chunk_prof.txt; exit 1; }
      grep -A22 "== CHUNK" gpurun_out/${TAG}_chunk_prof.txt | cut -c1-150 ;;
    abasync|abasync:*)
      V=0,0x1000000; [ "$step" != abasync ] && V="${step#abasync:}"
      timeout -k 10 400 python -u tools/ab_async.py --rounds 7 --steps 100 --variants "$V" > gpurun_out/${TAG}_ab_async.json 2> gpurun_out/${TAG}_ab_async.err || { tail -20 gpurun_out/${TAG}_ab_async.err; exit 1; }
      cat gpurun_out/${TAG}_ab_async.json ;;
    conf)
      timeout -k 10 300 python -u tools/conf_workload.py > gpurun_out/${TAG}_conf.json 2> gpurun_out/${TAG}_conf.err || { tail -20 gpurun_out/${TAG}_conf.err; exit 1; }
      cat gpurun_out/${TAG}_conf.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "steps done"
