# Calibrate the L2 -> fabric read counters on known-byte kernels (tools/fetch_calib.hip: streaming,
# one 4-byte word per line / half line / sector, integrate-like row gathers) and read the same
# counters on the integrate workload (tools/traffic_workload.py).  Two --pmc passes per program:
#   raw:   TCC_EA0_RDREQ, TCC_EA0_RDREQ_32B, TCC_BUBBLE, TCC_EA0_RDREQ_DRAM_32B (4 TCC slots)
#   fetch: FETCH_SIZE (3 TCC slots)
# Writes gpurun_out/calib/* and profiles/<round>_pmc_calib.json (tools/pmc_calib.py).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ROUND=${ROUND:-r03}
O=gpurun_out/calib
mkdir -p $O
timeout -k 10 60 tools/_ab/fetch_calib > $O/calib_plain.jsonl
RAW=TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum,TCC_BUBBLE_sum,TCC_EA0_RDREQ_DRAM_32B_sum
for pass in raw fetch; do
  [ $pass = raw ] && C=$RAW || C=FETCH_SIZE
  timeout -s KILL 90 rocprofv3 --pmc $(echo $C | tr , ' ') -d /tmp/cal_$pass -o cal --output-format csv -- tools/_ab/fetch_calib > $O/calib_$pass.jsonl 2> $O/calib_$pass.err
  cp "$(find /tmp/cal_$pass -name '*counter_collection.csv' | head -1)" $O/calib_${pass}_counters.csv
  timeout -s KILL 180 rocprofv3 --pmc $(echo $C | tr , ' ') -d /tmp/int_$pass -o int --output-format csv -- python3 tools/traffic_workload.py --out calib > $O/int_$pass.log 2>&1
  f="$(find /tmp/int_$pass -name '*counter_collection.csv' | head -1)"
  python3 -c "import pandas as pd,sys; d=pd.read_csv(sys.argv[1]); d[d['Kernel_Name'].str.contains('mqr::')].to_csv(sys.argv[2], index=False)" "$f" $O/int_${pass}_counters.csv
done
python3 tools/pmc_calib.py $O profiles/${ROUND}_pmc_calib.json
