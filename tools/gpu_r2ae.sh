# Round-2 GPU session AE: synth10k passes-per-task sweep (task front vs scan front: with fewer passes in flight
# the correlation's receiver reads can hit what the scan just streamed through the Infinity Cache).
set -o pipefail
mkdir -p gpurun_out/r2ae
for c in 8 4 2 1 16 8; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --chunk $c > gpurun_out/r2ae/c$c.json 2> gpurun_out/r2ae/c$c.err || { echo "chunk $c failed"; tail -5 gpurun_out/r2ae/c$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r2ae/c$c.json')); r=d['roofline']; print('chunk $c', round(d['value']), round(d['ms_per_step'],2), 'stack launch', round(r['launch_ms'],3), 'frac', round(r['frac'],3))"
done
