# Round-2 GPU session J: every workload's bench line (no CPU baseline) for the DESIGN tables.
set -o pipefail
mkdir -p gpurun_out/r2j
for wl in weights speeds sliding; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r2j/$wl.json 2> gpurun_out/r2j/$wl.err || { echo "$wl failed"; tail -5 gpurun_out/r2j/$wl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2j/$wl.json')); print('$wl', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_breakdown_ms'].items()}, round(d['roofline']['frac'],3), round(d['roofline']['launch_ms'],3))"
done
timeout -k 10 300 python bench.py --workload synth10k --scaling strong --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/r2j/synth10k_strong.json 2> gpurun_out/r2j/strong.err || { echo "strong failed"; tail -5 gpurun_out/r2j/strong.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2j/synth10k_strong.json')); print('synth10k strong', round(d['value']), round(d['ms_per_step'],3), d['scaling'])"
