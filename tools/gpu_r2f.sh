# Round-2 GPU session F: the whole -m gpu suite, then the default bench on both workloads.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/f_summary.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/f_tests.log 2>&1; rc=$?
echo tests=$rc; tail -8 gpurun_out/f_tests.log
[ $rc -eq 0 ] || exit 1
summ() { python -c "import json,sys; d=json.load(open('$1')); b=d['step_breakdown_ms']; print('$2', round(d['value']), 'step', round(d['ms_per_step'],2), {k: round(v,2) for k,v in b.items()}, 'frac', round(d['roofline']['frac'],3), 'corr', round(d['roofline']['correlation_frac'],3))"; }
for wl in synth10k weights; do
  timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 4 --warmup 1 > gpurun_out/f_$wl.json 2> gpurun_out/f.err || { echo "$wl failed"; tail -5 gpurun_out/f.err; exit 1; }
  summ gpurun_out/f_$wl.json "$wl" | tee -a gpurun_out/f_summary.txt
done
