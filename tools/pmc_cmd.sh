# SQ counter passes (one rocprofv3 --pmc run each, kernel trace only) over any command; per-dispatch averages of
# the kernels whose names contain FILTER -> gpurun_out/pmcc_<tag>.json
#     bash tools/pmc_cmd.sh TAG FILTER -- python bench.py --workload prep --steps 3 --no-cpu-baseline
set -o pipefail
tag=$1; filt=$2; shift 2; [ "$1" = "--" ] && shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/pmcc_$tag; rm -rf $d; mkdir -p $d
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $d/p$i -o pmc --output-format csv -- "$@" > /dev/null 2> $d/p$i.err \
    || { echo "pmc pass $i failed"; tail -3 $d/p$i.err; exit 1; }
done
python - "$d" "$filt" << 'PY'
import csv, glob, json, sys
from collections import defaultdict
d, filt = sys.argv[1], sys.argv[2]
per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if filt not in row["Kernel_Name"]:
            continue
        k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("dvh::", "")[:60]
        per[k][row["Counter_Name"]][(f, row["Dispatch_Id"])] += float(row["Counter_Value"])
res = {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in per.items()}
json.dump(res, open(d + ".json", "w"), indent=1)
for k, cs in res.items():
    print(k, " ".join("%s=%.4g" % (c, v) for c, v in sorted(cs.items())))
PY
rm -rf "$d"
