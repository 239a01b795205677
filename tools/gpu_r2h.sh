# Round-2 GPU session H: synth10k / weights with the validity as its own launch (scan alone vs correlation alone).
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/h_summary.txt
summ() { python -c "import json,sys; d=json.load(open('$1')); b=d['step_breakdown_ms']; print('$2', round(d['value']), 'step', round(d['ms_per_step'],2), {k: round(v,3) for k,v in b.items()}, 'frac', round(d['roofline']['frac'],3), d.get('validity_roofline'))"; }
for wl in synth10k weights; do
  for v in "--separate-validity" ""; do
    timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 4 --warmup 1 $v > gpurun_out/h.json 2> gpurun_out/h.err || { echo "$wl $v failed"; tail -5 gpurun_out/h.err; exit 1; }
    summ gpurun_out/h.json "$wl $v" | tee -a gpurun_out/h_summary.txt
  done
done
