"""Average per-dispatch PMC values of the hot-path kernels from rocprofv3 counter_collection CSVs.

    python tools/pmc_summary.py <dir with c*/ and p*/ .../*counter_collection.csv> <out.json>

Counter values are summed over the dimensions rocprofv3 reports per dispatch, then averaged over
the dispatches of each kernel.  HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB, and FETCH_SIZE is exact only after a per-access-width correction (gfx950
tallies wide streaming reads at half).  The correction is measured here, not assumed: the
calibration program tools/calib/fetch_calib streams 1 GiB with 4-byte-per-lane loads (the VSG
kernels' sub-window loads), 1 GiB with 16-byte-per-lane loads and 256 MiB of 4-byte float atomics;
"calibration" holds bytes / counter bytes for each, and every kernel's "traffic_bytes" is
FETCH_SIZE x the 4-byte read factor + WRITE_SIZE x the atomic factor (its stores are float atomics
and scratch).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ("vsg_stackv_kernel", "window_fixup_kernel", "vsg_stackf_kernel", "window_scan_kernel", "vsg_invalid_fill_kernel", "vsg_stack_kernel", "vsg_scales_kernel", "window_sumsq_kernel", "pass_geometry_kernel", "tdft_gemm_kernel", "tdft_rows_kernel", "fk_contract_kernel",
           "fv_kernel", "fv_batch_kernel", "fv_tile_kernel", "fv_mfma_kernel", "vsg_stackp_kernel", "vsg_gather_kernel",
           "sos_block_kernel", "sos_scan_kernel", "sos_transition_kernel", "row_stats_kernel", "impute_kernel",
           "row_normalize_kernel", "select_mean_kernel", "ridge_kernel", "read4", "read16", "atomic4")
CALIB_BYTES = {"read4": ("FETCH_SIZE", 1 << 30), "read16": ("FETCH_SIZE", 1 << 30), "atomic4": ("WRITE_SIZE", 256 << 20)}


def main():
    root, out = sys.argv[1], sys.argv[2]
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> value
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                k = next((k for k in KERNELS if k in name), None)
                if k is None:
                    continue
                disp = (f, row.get("Dispatch_Id", ""))
                per[k][row["Counter_Name"]][disp] += float(row["Counter_Value"])
    res = {}
    for k, ctrs in per.items():
        d = {}
        for c, v in ctrs.items():
            vals = list(v.values())
            d[c] = sum(vals) / len(vals)
            d[c + "_dispatches"] = len(vals)
        if "FETCH_SIZE" in d:
            d["fetch_bytes"] = d["FETCH_SIZE"] * 1024.0
            d["fetch_bytes_x2"] = 2 * d["fetch_bytes"]
        if "WRITE_SIZE" in d:
            d["write_bytes"] = d["WRITE_SIZE"] * 1024.0
        if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
            d["valu_per_wave"] = d["SQ_INSTS_VALU"] / max(d["SQ_WAVES"], 1)
        res[k] = d
    calib = {}
    for k, (ctr, nbytes) in CALIB_BYTES.items():
        if k in res and ctr in res[k] and res[k][ctr] > 0:
            calib[k] = nbytes / (res[k][ctr] * 1024.0)
    if calib:
        res["calibration"] = calib
        f4, fa = calib.get("read4"), calib.get("atomic4")
        for k, d in res.items():
            if k in CALIB_BYTES or k == "calibration" or f4 is None or fa is None:
                continue
            if "fetch_bytes" in d and "write_bytes" in d:
                d["traffic_bytes"] = d["fetch_bytes"] * f4 + d["write_bytes"] * fa
    lay = os.path.join(root, "layout.json")
    if os.path.exists(lay):  # the bench's launch layout these per-launch counters belong to
        res["layout"] = json.load(open(lay))
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(json.dumps({k: ({c: v for c, v in d.items() if not str(c).endswith("_dispatches")} if k != "layout" else d)
                      for k, d in res.items()}, indent=1))


if __name__ == "__main__":
    main()
