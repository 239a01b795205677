# SQ counter passes (one rocprofv3 --pmc run each, kernel trace only) over tools/exp_stack.py for one
# variant of the stack launch; per-dispatch averages -> gpurun_out/pmcx_<tag>.json
#     bash tools/pmc_exp.sh TAG corr|fused|corr7 [env assignments...]   (EXP_ARGS: extra exp_stack.py arguments)
set -o pipefail
tag=$1; only=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/pmcx_$tag; rm -rf $d; mkdir -p $d
i=0
groups=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
        "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH")
# PMC_GROUPS="G1;G2": other counter groups (each within one pass's limits)
[ -n "$PMC_GROUPS" ] && IFS=';' read -ra groups <<< "$PMC_GROUPS"
for grp in "${groups[@]}"; do
  i=$((i+1))
  env "$@" timeout -s KILL 120 rocprofv3 --pmc $grp -d $d/p$i -o pmc --output-format csv -- python tools/exp_stack.py --reps 3 --only $only $EXP_ARGS > /dev/null 2> $d/p$i.err || { echo "pmc pass $i failed"; tail -3 $d/p$i.err; exit 1; }
done
python - "$d" << 'PY'
import csv, glob, json, sys
from collections import defaultdict
d = sys.argv[1]
per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].split("<")[0].split()[-1][:60]
        if "vsg_stack" not in row["Kernel_Name"] and "sumsq" not in row["Kernel_Name"]:
            continue
        per[k][row["Counter_Name"]][(f, row["Dispatch_Id"])] += float(row["Counter_Value"])
res = {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in per.items()}
json.dump(res, open(d + ".json", "w"), indent=1)
for k, cs in res.items():
    print(k, " ".join("%s=%.4g" % (c, v) for c, v in sorted(cs.items())))
PY
rm -rf "$d"
