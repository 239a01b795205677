"""Average per-dispatch PMC values of the hot-path kernels from rocprofv3 counter_collection CSVs.

    python tools/pmc_summary.py <dir with p*/.../*counter_collection.csv> <out.json>

Counter values are summed over the dimensions rocprofv3 reports per dispatch, then averaged over
the dispatches of each kernel.  HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB; FETCH_SIZE is reported as-is and doubled ("fetch_bytes_x2") because gfx950
tallies 128-B requests at 64 B for wide streaming reads (the correction is calibrated only for
16-B-per-lane loads; our loads are 4 B per lane, so both figures are kept).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ("vsg_stackf_kernel", "vsg_stack_kernel", "vsg_scales_kernel", "tdft_gemm_kernel", "fk_contract_kernel",
           "fv_kernel")


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
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(json.dumps({k: {c: v for c, v in d.items() if not c.endswith("_dispatches")} for k, d in res.items()},
                     indent=1))


if __name__ == "__main__":
    main()
