# Round-2 GPU session E: the whole -m gpu suite, then bench with / without pivot tables.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/e_summary.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=20 > gpurun_out/e_tests.log 2>&1; rc=$?
echo tests=$rc; tail -45 gpurun_out/e_tests.log
[ $rc -eq 0 ] || exit 1
summ() { python -c "import json,sys; d=json.load(open('$1')); b=d['step_breakdown_ms']; print('$2', round(d['value']), 'step', round(d['ms_per_step'],2), {k: round(v,2) for k,v in b.items()}, 'frac', round(d['roofline']['frac'],3))"; }
for wl in synth10k weights; do
  for v in "" "--no-pivot-table"; do
    timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 4 --warmup 1 $v > gpurun_out/e.json 2> gpurun_out/e.err || { echo "$wl $v failed"; tail -5 gpurun_out/e.err; exit 1; }
    summ gpurun_out/e.json "$wl $v" | tee -a gpurun_out/e_summary.txt
  done
done
