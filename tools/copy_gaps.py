"""Timeline of the host-fed step's H2D copies from a rocprofv3 --memory-copy-trace run (this rocprofv3 records no
byte counts, so the staging chunks are told by their duration, >= 0.3 ms): the copy engine's busy time, the span
from the first to the last chunk, and the gaps between chunks (the host-side bubbles between and inside the
classes' get_images calls).      python tools/copy_gaps.py <rocprofv3 output dir>
"""
import csv
import glob
import sys

d = sys.argv[1]
h2d = []
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "HOST_TO_DEVICE" in r.get("Direction", ""):
            h2d.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
h2d.sort()
big = [c for c in h2d if c[1] - c[0] >= 300_000]
if not big:
    sys.exit("no staging chunks found")
busy = sum(e - s for s, e in big)
span = big[-1][1] - big[0][0]
gaps = [(s1 - e0) for (s0, e0), (s1, e1) in zip(big, big[1:])]
print("chunks %d  busy %.2f ms  span %.2f ms  gaps > 0.1 ms: %d totalling %.2f ms" % (
    len(big), busy / 1e6, span / 1e6, sum(g > 100_000 for g in gaps), sum(g for g in gaps if g > 100_000) / 1e6))
print("gaps (ms):", " ".join("%.2f" % (g / 1e6) for g in gaps if g > 100_000))
