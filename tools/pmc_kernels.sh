#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run per group, each under its own time limit) over
# tools/traffic_workload.py, reduced to per-launch means for kernels matching $1.
# Usage (on the box): bash tools/pmc_kernels.sh '<kernel regex>' [workload args...]
set -o pipefail
RE="$1"; shift
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
G2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
i=0
for G in "$G1" "$G2"; do
  i=$((i+1))
  rm -rf /tmp/pmck/p$i
  timeout -s KILL 120 rocprofv3 --pmc $G -d /tmp/pmck/p$i -o p --output-format csv -- \
    python3 tools/traffic_workload.py --out pmck "$@" > gpurun_out/pmck_p$i.log 2>&1 || { tail -5 gpurun_out/pmck_p$i.log; exit 1; }
done
python3 - "$RE" <<'PY'
import glob, re, sys, json
import pandas as pd
rx = re.compile(sys.argv[1])
res = {}
for path in glob.glob("/tmp/pmck/**/*counter_collection.csv", recursive=True):
    df = pd.read_csv(path)
    df = df[df["Kernel_Name"].map(lambda n: bool(rx.search(n)))]
    for (k, c), g in df.groupby(["Kernel_Name", "Counter_Name"]):
        short = k.split("(")[0][-60:]
        res.setdefault(short, {})[c] = float(g["Counter_Value"].mean())
        res[short]["launches"] = int(len(g))
with open("gpurun_out/pmck_summary.json", "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res, indent=1))
PY
