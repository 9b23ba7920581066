# SQ instruction/cycle counters of the integrate kernel for a few variants (rocprofv3 --pmc, one
# counter group per pass); the csv passes are reduced on the box to gpurun_out/sq_summary.jsonl.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
: > gpurun_out/sq_summary.jsonl
for v in ${VARIANTS:-0 11 13}; do
  d=/tmp/sq_v$v
  timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES -d $d/a -o a --output-format csv -- python3 tools/traffic_workload.py --variant $v --out sq_v$v > gpurun_out/sq_v$v.log 2>&1
  timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $d/b -o b --output-format csv -- python3 tools/traffic_workload.py --variant $v --out sq_v$v >> gpurun_out/sq_v$v.log 2>&1
  cp gpurun_out/sq_v$v/workload.json $d/
  python3 tools/sq_summary.py $d >> gpurun_out/sq_summary.jsonl
done
