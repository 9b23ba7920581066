#!/bin/bash
# Counter passes (one rocprofv3 --pmc run per group, each under its own time limit) over
# tools/traffic_workload.py, reduced to per-launch means for kernels matching $1.
# Groups come from $PMC_GROUPS (';'-separated); the output name from $PMC_OUT (default pmcg).
# Usage (on the box): PMC_GROUPS="A B;C D" bash tools/pmc_groups.sh '<kernel regex>' [workload args...]
set -o pipefail
RE="$1"; shift
OUT="${PMC_OUT:-pmcg}"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf /tmp/$OUT
IFS=';' read -ra GROUPS_ <<< "$PMC_GROUPS"
i=0
for G in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G -d /tmp/$OUT/p$i -o p --output-format csv -- \
    python3 tools/traffic_workload.py --out $OUT "$@" > gpurun_out/${OUT}_p$i.log 2>&1 || { tail -5 gpurun_out/${OUT}_p$i.log; exit 1; }
done
python3 - "$RE" "$OUT" <<'PY'
import glob, re, sys, json
import pandas as pd
rx = re.compile(sys.argv[1])
res = {}
for path in glob.glob(f"/tmp/{sys.argv[2]}/**/*counter_collection.csv", recursive=True):
    df = pd.read_csv(path)
    df = df[df["Kernel_Name"].map(lambda n: bool(rx.search(n)))]
    for (k, c), g in df.groupby(["Kernel_Name", "Counter_Name"]):
        short = k.split("(")[0][-60:]
        res.setdefault(short, {})[c] = float(g["Counter_Value"].mean())
        res[short]["launches"] = int(len(g))
with open(f"gpurun_out/{sys.argv[2]}_summary.json", "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res, indent=1))
PY
