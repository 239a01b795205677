"""Per-dispatch FETCH_SIZE of the validated stack launch for two variant libraries (gpurun_out/pmcab_<v>/):
the HBM read bytes an A/B changes (x 2: gfx950 tallies 16-byte streaming reads at half, MI355X_MICROARCH.md)."""
import csv
import glob

for v in ("base", "skip"):
    tot = {}
    for f in glob.glob(f"gpurun_out/pmcab_{v}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            if "stackv" in k or "zero_fixup" in k:
                key = (k[:40], row.get("Dispatch_Id"))
                tot[key] = tot.get(key, 0.0) + float(row.get("Counter_Value", 0))
    vals = {}
    for (k, d), x in tot.items():
        vals.setdefault(k, []).append(x)
    for k, xs in vals.items():
        print(v, k, len(xs), "FETCH_SIZE KiB/dispatch", round(sum(xs) / len(xs)), "~ GB (x2):",
              round(2 * 1024 * sum(xs) / len(xs) / 1e9, 3))
