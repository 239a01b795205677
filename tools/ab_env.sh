# A/B of run-time switches on the bench (run on the box through gpurun):
#   bash tools/ab_env.sh TAG "ENV1=a ENV2=b" "ENV1=c" ... -- bench args
# each variant's bench line -> gpurun_out/ab_TAG_<k>.json, one summary line per variant, two rounds (ABAB order)
set -o pipefail
tag=$1; shift
vars=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do vars+=("$1"); shift; done; [ "$1" = "--" ] && shift
mkdir -p gpurun_out
for r in 1 2; do
  for k in "${!vars[@]}"; do
    out=gpurun_out/ab_${tag}_${k}_$r.json
    env ${vars[$k]} timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$out" 2> "${out%.json}.err" \
      || { echo "variant $k failed"; tail -5 "${out%.json}.err"; exit 1; }
    python - "$out" "${vars[$k]}" << 'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d.get("roofline") or {}
print("%-28s value %.0f  ms/step %.3f  launch %.3f ms  frac %.3f" % (sys.argv[2], d["value"], d["ms_per_step"],
      r.get("launch_ms", 0), r.get("frac", 0)))
PY
  done
done
