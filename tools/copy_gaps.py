"""Timeline of the host-fed step's H2D copies from a rocprofv3 --memory-copy-trace --kernel-trace run: busy time of
the copy engine, the span from the first to the last copy, and the gaps between copies with the kernels that ran
in them.      python tools/copy_gaps.py <rocprofv3 output dir>
"""
import csv
import glob
import sys

d = sys.argv[1]
copies, kernels = [], []
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if not copies and not kernels:
            print("columns:", list(r.keys()))
        kind = " ".join(str(v) for k, v in r.items() if k in ("Direction", "Operation", "Kind"))
        size = next((int(float(v)) for k, v in r.items() if ("Size" in k or "Bytes" in k) and v), 0)
        if "HOST_TO_DEVICE" in kind or "H2D" in kind or "HostToDevice" in kind:
            copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), size))
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        kernels.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
copies.sort()
kernels.sort()
big = [c for c in copies if c[2] >= (8 << 20)]
print("copies", len(copies), ">= 8 MB", len(big))
if big:
    busy = sum(e - s for s, e, _ in big)
    nbytes = sum(b for _, _, b in big)
    print("busy %.2f ms for %.2f GB = %.1f GB/s" % (busy / 1e6, nbytes / 1e9, nbytes / busy))
    gaps = []
    for (s0, e0, _), (s1, e1, _) in zip(big, big[1:]):
        if s1 - e0 > 100_000:
            ks = [k for k in kernels if k[0] >= e0 and k[1] <= s1]
            gaps.append((s1 - e0, e0, [k[2] for k in ks][:4]))
    print("gaps > 0.1 ms:", len(gaps), "total %.2f ms" % (sum(g[0] for g in gaps) / 1e6))
    for g, t, ks in gaps[:40]:
        print("  %.2f ms at +%.1f ms  kernels: %s" % (g / 1e6, (t - big[0][0]) / 1e6, ks))
