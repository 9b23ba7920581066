#!/bin/bash
# HBM traffic A/B of integrate variants: FETCH_SIZE and WRITE_SIZE passes of tools/traffic_workload.py
# per variant (each pass under its own time limit), summarised by tools/pmc_summary.py into
# gpurun_out/traffic_v<variant>.json.  Usage (on the box): VARIANTS="-1 32768" bash tools/traffic_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in ${VARIANTS:--1}; do
  d=gpurun_out/tab_v$v
  mkdir -p $d
  for c in FETCH_SIZE WRITE_SIZE; do
    n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    rm -rf /tmp/tab_$n
    timeout -s KILL 180 rocprofv3 --pmc $c -d /tmp/tab_$n -o $n --output-format csv -- \
      python3 tools/traffic_workload.py --variant $v --out tab_v$v > $d/$n.log 2>&1 || { tail -5 $d/$n.log; exit 1; }
    f=$(find /tmp/tab_$n -name "*counter_collection.csv" | head -1)
    python3 -c "import pandas as pd,sys; d=pd.read_csv(sys.argv[1]); d[d['Kernel_Name'].str.contains('mqr::')].to_csv(sys.argv[2], index=False)" $f $d/${n}_counter_collection.csv
  done
  python3 tools/pmc_summary.py $d gpurun_out/traffic_v$v.json > $d/summary.log || exit 1
  grep -E "traffic_over_alg|traffic_bytes_per_launch" gpurun_out/traffic_v$v.json
done
