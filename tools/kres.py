"""Register / scratch / occupancy of every kernel in a HIP source (hipcc -Rpass-analysis=kernel-resource-usage).

    python tools/kres.py das_diff_veh_amd/csrc/dvh_vsg.hip [-DNAME=1 ...] [--grep stackv]
"""
import re
import subprocess
import sys

args = sys.argv[1:]
grep = None
if "--grep" in args:
    i = args.index("--grep")
    grep = args[i + 1]
    del args[i:i + 2]
src, defs = args[0], args[1:]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics",
       "-fno-slp-vectorize", "-Idas_diff_veh_amd/csrc", "-Iinclude", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage", *defs]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        cur = {"name": re.sub(r"\(.*", "", dm).replace("dvh::", "")}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if grep and grep not in r["name"]:
        continue
    print(f"{r['name'][:90]:90s} vgpr {r.get('VGPRs','?'):>4} agpr {r.get('AGPRs','?'):>4} "
          f"scratch {r.get('ScratchSize [bytes/lane]','?'):>4} occ {r.get('Occupancy [waves/SIMD]','?'):>2} "
          f"lds {r.get('LDS Size [bytes/block]','?')}")
