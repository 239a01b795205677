# Round-2 GPU session L: A/B of stack-launch switches (receiver nt loads, correlation priority, scan depth).
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/l_summary.txt
summ() { python -c "import json,sys; d=json.load(open('$1')); b=d['step_breakdown_ms']; print('$2', round(d['value']), 'step', round(d['ms_per_step'],2), 'stack', round(b['stack'],3), 'frac', round(d['roofline']['frac'],3))"; }
for v in ${VARIANTS:-default rcvnt prio2 ntprio d12 default}; do
  lib=""; [ $v = default ] || lib=das_diff_veh_amd/lib/variants/$v.so
  for wl in synth10k weights sliding; do
    DVH_LIB=$lib timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 4 --warmup 1 > gpurun_out/l.json 2> gpurun_out/l.err || { echo "$v $wl failed"; tail -5 gpurun_out/l.err; exit 1; }
    summ gpurun_out/l.json "$v $wl" | tee -a gpurun_out/l_summary.txt
  done
done
