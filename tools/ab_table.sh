# A/B of pivot-table variants: bench (fused + separate validity, with / without table) per library.
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.load(open('$1')); b=d['step_breakdown_ms']; print('$2', round(d['value']), 'step', round(d['ms_per_step'],2), 'stack', round(b['stack'],2), 'frac', round(d['roofline']['frac'],3))"; }
for v in ${VARIANTS:-default}; do
  lib=""; [ $v = default ] || lib=das_diff_veh_amd/lib/variants/$v.so
  for wl in synth10k weights; do
    for o in "" "--separate-validity" "--separate-validity --no-pivot-table"; do
      DVH_LIB=$lib timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 4 --warmup 1 $o > gpurun_out/abt.json 2> gpurun_out/abt.err || { echo "$v $wl $o failed"; tail -5 gpurun_out/abt.err; exit 1; }
      summ gpurun_out/abt.json "$v $wl $o"
    done
  done
done
