# Quick PMC look at one workload's kernels (2 counter passes + FETCH/WRITE), summary to stdout.
#   bash tools/pmc_quick.sh <workload> [extra bench args]
set -o pipefail
wl=${1:-synth10k}; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
d=gpurun_out/pmcq_$wl; rm -rf $d; mkdir -p $d
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -d $d/p$i -o pmc --output-format csv -- python bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline "$@" > /dev/null 2> $d/p$i.err || { echo "pmc pass $i failed"; tail -3 $d/p$i.err; exit 1; }
done
python tools/pmc_summary.py $d $d/summary.json > /dev/null && python - "$d/summary.json" << 'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if k in ("layout", "calibration"):
        continue
    keys = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
            "SQ_ACTIVE_INST_VALU", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS", "SQ_INSTS_VMEM_RD", "SQ_WAIT_INST_LDS",
            "TCC_HIT_sum", "TCC_MISS_sum", "fetch_bytes", "write_bytes"]
    print(k, {c: round(v[c] / 1e6, 2) for c in keys if c in v}, "(millions)")
PY
