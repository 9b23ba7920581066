#!/usr/bin/env python3
"""Summarise tools/pmc_calib.sh: per kernel, the read bytes each counter formula implies, divided by
the kernel's known distinct-line bytes (fetch_calib) or by the integrate kernel's algorithmic bytes.

  fetch_size   FETCH_SIZE (KiB, rocprofv3's gfx950 formula)
  req64        64 x TCC_EA0_RDREQ (every request tallied as 64 B)
  formula      128 BUBBLE + 64 (RDREQ - BUBBLE - RDREQ_32B) + 32 RDREQ_32B (= FETCH_SIZE by definition)
  dram32       32 x TCC_EA0_RDREQ_DRAM_32B (width-aware: a 64-B request counts 2, 128-B counts 4)

Usage: pmc_calib.py <dir> <out.json>"""
import json
import sys

import pandas as pd


def per_dispatch(path):
    d = pd.read_csv(path)
    d["k"] = d["Kernel_Name"].str.extract(r"(k_\w+)")
    # sum over any per-instance rows, then one row per dispatch
    return d.pivot_table(index=["Dispatch_Id", "k"], columns="Counter_Name", values="Counter_Value", aggfunc="sum")


def bytes_of(row):
    g = lambda c: float(row.get(c, float("nan")))
    R, S, B, D = g("TCC_EA0_RDREQ_sum"), g("TCC_EA0_RDREQ_32B_sum"), g("TCC_BUBBLE_sum"), g("TCC_EA0_RDREQ_DRAM_32B_sum")
    return {"rdreq": R, "rdreq_32b": S, "bubble": B, "dram_32b": D, "req64": 64 * R,
            "formula": 128 * B + 64 * (R - B - S) + 32 * S, "dram32": 32 * D}


def main(d, out):
    rec = {"calibration": [], "integrate": None}
    plain = [json.loads(l) for l in open(f"{d}/calib_raw.jsonl")]
    raw = per_dispatch(f"{d}/calib_raw_counters.csv").reset_index()
    fet = per_dispatch(f"{d}/calib_fetch_counters.csv").reset_index()
    # fetch_calib launches, per rep: (flush, measured) x 5; rep 1 (the second) is the record
    raw, fet = raw.sort_values("Dispatch_Id"), fet.sort_values("Dispatch_Id")
    measured_raw = raw.iloc[1::2].reset_index(drop=True)
    measured_fet = fet.iloc[1::2].reset_index(drop=True)
    for i, p in enumerate(plain):
        if i < len(plain) // 2:
            continue
        b = bytes_of(measured_raw.iloc[i])
        b["fetch_size"] = 1024.0 * float(measured_fet.iloc[i]["FETCH_SIZE"])
        lb = p["line_bytes"]
        rec["calibration"].append({"kernel": p["kernel"], "line_bytes": lb, "ms": p["ms"],
                                   **{f"{k}_over_line_bytes": b[k] / lb for k in ("fetch_size", "req64", "formula", "dram32")},
                                   "counters": {k: b[k] for k in ("rdreq", "rdreq_32b", "bubble", "dram_32b")}})
    wl = json.load(open(f"{d}/workload.json"))
    ir = per_dispatch(f"{d}/int_raw_counters.csv")
    ifz = per_dispatch(f"{d}/int_fetch_counters.csv")
    ik = [k for k in ir.index.get_level_values("k").unique() if str(k).startswith("k_integrate")]
    ik = max(ik, key=lambda k: ir.xs(k, level="k")["TCC_EA0_RDREQ_sum"].mean())
    row = ir.xs(ik, level="k").mean()
    b = bytes_of(row)
    b["fetch_size"] = 1024.0 * float(ifz.xs(ik, level="k")["FETCH_SIZE"].mean())
    alg = wl["alg_bytes_total"] / wl["integrate_launches"]
    rec["integrate"] = {"kernel": ik, "alg_read_write_bytes_per_launch": alg,
                        **{f"{k}_read_bytes_per_launch": b[k] for k in ("fetch_size", "req64", "formula", "dram32")},
                        "counters": {k: b[k] for k in ("rdreq", "rdreq_32b", "bubble", "dram_32b")}, "workload": wl}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
