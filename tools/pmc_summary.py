#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/traffic_workload.py into a traffic record.

FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters).  They are calibrated on k_pack,
whose bytes are known exactly and whose accesses have the same width (8 B/lane float2) as the
integrate kernel's voxel loads/stores: traffic = FETCH * (pack_read / FETCH_pack) +
WRITE * (pack_write / WRITE_pack).  Output: profiles/<name>.json."""
import json
import sys

import pandas as pd


def per_kernel(path, counter):
    d = pd.read_csv(path)
    d = d[d["Counter_Name"] == counter]
    d["k"] = d["Kernel_Name"].str.extract(r"(k_\w+)")
    return d.groupby("k")["Counter_Value"].agg(["mean", "sum", "count"])


def main(pmc_dir, out):
    wl = json.load(open(f"{pmc_dir}/workload.json"))
    fetch = per_kernel(f"{pmc_dir}/fetch_counter_collection.csv", "FETCH_SIZE")
    write = per_kernel(f"{pmc_dir}/write_counter_collection.csv", "WRITE_SIZE")
    kr = wl["pack_read_bytes"] / (fetch.loc["k_pack", "sum"] * 1024.0)
    kw = wl["pack_write_bytes"] / (write.loc["k_pack", "sum"] * 1024.0)
    # the dominant integrate kernel (the lean default is followed by an exact fix-up launch that
    # normally exits at once)
    ik = max((k for k in fetch.index if k.startswith("k_integrate")), key=lambda k: fetch.loc[k, "mean"])
    n = fetch.loc[ik, "count"]
    raw_r = fetch.loc[ik, "mean"] * 1024.0
    raw_w = write.loc[ik, "mean"] * 1024.0
    tk = next((k for k in fetch.index if k.startswith("k_touch")), None)
    rec = {"kernel": ik, "launches": int(n),
           "fetch_bytes_per_launch_raw": raw_r, "write_bytes_per_launch_raw": raw_w,
           "read_calibration": kr, "write_calibration": kw,
           "traffic_bytes_per_launch": raw_r * kr + raw_w * kw,
           "alg_bytes_per_launch": wl["alg_bytes_total"] / wl["integrate_launches"],
           "touch_fetch_bytes_per_launch_raw": float(fetch.loc[tk, "mean"] * 1024.0) if tk else None,
           "integrate_src": wl.get("integrate_src"), "variant_ran": wl.get("variant_ran"),
           "workload": wl}
    rec["traffic_over_alg"] = rec["traffic_bytes_per_launch"] / rec["alg_bytes_per_launch"]
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
