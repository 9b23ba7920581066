#!/bin/bash
# Counter passes over the confidence kernel (tools/conf_workload.py), one rocprofv3 --pmc run per
# group under its own time limit; per-launch means of k_confidence -> gpurun_out/pmc_conf.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1 || true
GROUPS_=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD TA_BUSY_avr GRBM_GUI_ACTIVE"
         "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE")
i=0
for G in "${GROUPS_[@]}"; do
  i=$((i+1))
  rm -rf /tmp/pmcconf/p$i
  timeout -s KILL 120 rocprofv3 --pmc $G -d /tmp/pmcconf/p$i -o p --output-format csv -- \
    python3 tools/conf_workload.py > gpurun_out/pmcconf_p$i.log 2>&1 || { echo "group $i failed"; tail -3 gpurun_out/pmcconf_p$i.log; }
done
python3 - <<'PY'
import glob, json
import pandas as pd
res = {}
for path in glob.glob("/tmp/pmcconf/**/*counter_collection.csv", recursive=True):
    df = pd.read_csv(path)
    df = df[df["Kernel_Name"].str.contains("k_confidence")]
    for c, g in df.groupby("Counter_Name"):
        res[c] = float(g["Counter_Value"].mean())
        res.setdefault("launches", int(len(g)))
        res.setdefault("duration_ns", float((g["End_Timestamp"] - g["Start_Timestamp"]).mean()))
try:
    res["confidence_src"] = json.load(open("gpurun_out/conf_workload.json")).get("confidence_src")
except (OSError, ValueError):
    res["confidence_src"] = None
cyc = res.get("GRBM_GUI_ACTIVE", 0.0) / 8
if cyc:
    f64 = sum(res.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                         "SQ_INSTS_VALU_TRANS_F64"))
    v = res.get("SQ_INSTS_VALU", 0.0)
    res["derived"] = {"gpu_cycles": cyc, "clock_ghz": cyc / res["duration_ns"],
                      # wave64 VALU: 2 cycles on a SIMD-32 (1024 SIMDs); f64 at half the f32 rate: 4
                      "valu_issue_frac_f32_rate": 2.0 * v / 1024 / cyc,
                      "valu_issue_frac_f64_at_half_rate": (2.0 * (v - f64) + 4.0 * f64) / 1024 / cyc,
                      "f64_share_of_valu": f64 / v if v else None,
                      "ta_busy_frac": res.get("TA_BUSY_avr", 0) / cyc if "TA_BUSY_avr" in res else None,
                      # resident waves per SIMD over the launch: SQ_WAVE_CYCLES counts quad-cycles
                      # (MI355X_MICROARCH.md), / (1024 SIMDs x cycles)
                      "waves_per_simd": 4.0 * res.get("SQ_WAVE_CYCLES", 0.0) / 1024 / cyc if "SQ_WAVE_CYCLES" in res else None}
json.dump(res, open("gpurun_out/pmc_conf.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
grep -i "f64\|FP64" gpurun_out/pmc_avail.txt | head -20 || true
