#!/bin/bash
# Counter comparison of integrate-kernel variants (one rocprofv3 --pmc pass per counter group and
# variant, each under its own time limit) over tools/traffic_workload.py; per-launch means of the
# kernels matching $KRE go to gpurun_out/pmc_ab.json.  Usage (on the box):
#   VARIANTS="0 3" bash tools/pmc_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
KRE="${KRE:-k_integrate_(wt|win|lean|lt|pk)}"
GROUPS_=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
         "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE")
for v in ${VARIANTS:-0 3}; do
  i=0
  for G in "${GROUPS_[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $G -d /tmp/pmcab/v$v/p$i -o p --output-format csv -- \
      python3 tools/traffic_workload.py --variant $v --out pmcab_v$v > gpurun_out/pmcab_v${v}_p$i.log 2>&1 || { tail -5 gpurun_out/pmcab_v${v}_p$i.log; exit 1; }
  done
done
python3 - "$KRE" <<'PY'
import glob, re, sys, json
import pandas as pd
rx = re.compile(sys.argv[1])
res = {}
for path in glob.glob("/tmp/pmcab/**/*counter_collection.csv", recursive=True):
    var = re.search(r"/v(\d+)/", path).group(1)
    df = pd.read_csv(path)
    df = df[df["Kernel_Name"].map(lambda n: bool(rx.search(n)))]
    for (k, c), g in df.groupby(["Kernel_Name", "Counter_Name"]):
        short = "v" + var + ":" + k.split("(")[0][-40:]
        res.setdefault(short, {})[c] = float(g["Counter_Value"].mean())
        res[short]["launches"] = int(len(g))
        if "Start_Timestamp" in g:
            res[short].setdefault("duration_ns_per_pass", []).append(
                float((g["End_Timestamp"] - g["Start_Timestamp"]).mean()))
# the build each variant's passes measured (tools/traffic_workload.py --out pmcab_v<var>)
for short, r in res.items():
    try:
        wl = json.load(open(f"gpurun_out/pmcab_v{short[1:].split(':')[0]}/workload.json"))
        r["integrate_src"], r["variant_ran"] = wl.get("integrate_src"), wl.get("variant_ran")
    except (OSError, ValueError):
        pass
# derived per-launch rates: fraction of the launch's GPU cycles each unit was busy.  GRBM_GUI_ACTIVE
# is summed over the 8 XCDs' graphics blocks: cycles of the launch = GRBM_GUI_ACTIVE / 8 (checked
# against the pass's own kernel duration: ~2.2 GHz under this load).
for r in res.values():
    cyc = r.get("GRBM_GUI_ACTIVE", 0.0) / 8
    if cyc:
        r["derived"] = {
            "gpu_cycles": cyc,
            "clock_ghz": cyc / (sum(r["duration_ns_per_pass"]) / len(r["duration_ns_per_pass"])),
            "ta_busy_frac": r.get("TA_BUSY_avr", 0.0) / cyc,
            "tcp_lookups_per_cu_cycle": r.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0.0) / 256 / cyc,
            "valu_issue_frac": 2.0 * r.get("SQ_INSTS_VALU", 0.0) / 1024 / cyc,  # wave64 VALU: 2 cycles on a SIMD-32
            "lds_insts": r.get("SQ_INSTS_LDS"),
        }
with open("gpurun_out/pmc_ab.json", "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res, indent=1))
PY
