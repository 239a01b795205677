# A/B of the validated stack launch configurations (variant libraries under das_diff_veh_amd/lib/variants).
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.load(open('$1')); b=d['step_breakdown_ms']; print('$2', round(d['value']), 'step', round(d['ms_per_step'],2), 'stack', round(b['stack'],2), 'scales', round(b['scales'],2), 'frac', round(d['roofline']['frac'],3))"; }
for v in ${VARIANTS:-default rcv2 rcv2d24}; do
  lib=""; [ $v = default ] || lib=das_diff_veh_amd/lib/variants/$v.so
  for wl in synth10k weights; do
    DVH_LIB=$lib timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 4 --warmup 1 > gpurun_out/ab_${v}_$wl.json 2> gpurun_out/ab_${v}_$wl.err || { echo "$v $wl failed"; tail -5 gpurun_out/ab_${v}_$wl.err; exit 1; }
    summ gpurun_out/ab_${v}_$wl.json "$v $wl"
  done
done
