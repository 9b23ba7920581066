#!/bin/bash
# Counter passes over the extraction kernels (tools/ab_extract.py, the bench's C2 mesh at 1.5), one
# rocprofv3 --pmc run per group under its own time limit; per-launch means per kernel ->
# gpurun_out/pmc_extract.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
GROUPS_=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD TA_BUSY_avr GRBM_GUI_ACTIVE")
i=0
for G in "${GROUPS_[@]}"; do
  i=$((i+1))
  rm -rf /tmp/pmcex/p$i
  timeout -s KILL 120 rocprofv3 --pmc $G -d /tmp/pmcex/p$i -o p --output-format csv -- \
    python3 tools/ab_extract.py --modes 0 --reps 5 > gpurun_out/pmcex_p$i.log 2>&1 || { echo "group $i failed"; tail -3 gpurun_out/pmcex_p$i.log; exit 1; }
done
python3 - <<'PY'
import glob, json
import pandas as pd
res = {}
for path in glob.glob("/tmp/pmcex/**/*counter_collection.csv", recursive=True):
    df = pd.read_csv(path)
    for kname in ("k_mc_bits", "k_mc_count", "k_mc_emit", "k_scan_counts"):
        d = df[df["Kernel_Name"].str.contains(kname)]
        if d.empty:
            continue
        r = res.setdefault(kname, {})
        for c, g in d.groupby("Counter_Name"):
            r[c] = float(g["Counter_Value"].mean())
        r.setdefault("launches", int(d["Dispatch_Id"].nunique()) if "Dispatch_Id" in d else None)
        r.setdefault("duration_ns", float((d["End_Timestamp"] - d["Start_Timestamp"]).mean()))
for k, r in res.items():
    cyc = r.get("GRBM_GUI_ACTIVE", 0.0) / 8
    if cyc:
        v = r.get("SQ_INSTS_VALU", 0.0)
        r["derived"] = {"gpu_cycles": cyc, "valu_issue_frac": 2.0 * v / 1024 / cyc,
                        "waves_per_simd": 4.0 * r.get("SQ_WAVE_CYCLES", 0.0) / 1024 / cyc if "SQ_WAVE_CYCLES" in r else None,
                        "wait_frac_of_wave_cycles": r["SQ_WAIT_ANY"] / r["SQ_WAVE_CYCLES"] if "SQ_WAIT_ANY" in r and r.get("SQ_WAVE_CYCLES") else None,
                        "ta_busy_frac": r.get("TA_BUSY_avr", 0) / cyc if "TA_BUSY_avr" in r else None}
json.dump(res, open("gpurun_out/pmc_extract.json", "w"), indent=1)
print(json.dumps({k: (r.get("duration_ns"), r.get("derived")) for k, r in res.items()}, indent=1))
PY
