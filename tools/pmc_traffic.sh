# HBM traffic of the integrate kernel (FETCH_SIZE / WRITE_SIZE, separate --pmc passes, calibrated
# on k_pack by tools/pmc_summary.py).  Writes gpurun_out/pmc/{fetch,write}_counter_collection.csv
# (filtered to the library's kernels) and profiles/<round>_pmc_traffic.json.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ROUND=${ROUND:-r02}
mkdir -p gpurun_out/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -k 10 180 rocprofv3 --pmc $c -d /tmp/pmc_$n -o $n --output-format csv -- python3 tools/traffic_workload.py > gpurun_out/pmc/$n.log 2>&1
  f=$(find /tmp/pmc_$n -name "*counter_collection.csv" | head -1)
  python3 -c "import pandas as pd,sys; d=pd.read_csv(sys.argv[1]); d[d['Kernel_Name'].str.contains('mqr::')].to_csv(sys.argv[2], index=False)" $f gpurun_out/pmc/${n}_counter_collection.csv
done
python3 tools/pmc_summary.py gpurun_out/pmc profiles/${ROUND}_pmc_traffic.json > gpurun_out/pmc/summary.log
cp gpurun_out/pmc/fetch_counter_collection.csv profiles/${ROUND}_pmc_fetch.csv
cp gpurun_out/pmc/write_counter_collection.csv profiles/${ROUND}_pmc_write.csv
