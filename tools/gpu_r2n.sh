# Round-2 GPU session N: the whole -m gpu suite, then sliding merged vs per-batch launches and the
# cross-pass prefetch variant.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/n_summary.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/n_tests.log 2>&1; rc=$?
echo tests=$rc; tail -4 gpurun_out/n_tests.log
[ $rc -eq 0 ] || exit 1
summ() { python -c "import json,sys; d=json.load(open('$1')); b=d['step_breakdown_ms']; print('$2', round(d['value']), 'step', round(d['ms_per_step'],2), {k: round(v,2) for k,v in b.items()}, 'frac', round(d['roofline']['frac'],3), 'launch', round(d['roofline']['launch_ms'],3))"; }
for m in 49 7 1; do
  timeout -k 10 300 python bench.py --workload sliding --no-cpu-baseline --steps 5 --warmup 1 --sliding-merge $m > gpurun_out/n.json 2> gpurun_out/n.err || { echo "merge $m failed"; tail -5 gpurun_out/n.err; exit 1; }
  summ gpurun_out/n.json "sliding merge $m" | tee -a gpurun_out/n_summary.txt
done
VARIANTS="default xpf" bash tools/gpu_r2l.sh
for v in default vt8; do
  lib=""; [ $v = default ] || lib=das_diff_veh_amd/lib/variants/$v.so
  DVH_LIB=$lib timeout -k 10 200 python tools/bench_timelapse.py > gpurun_out/n_tl.json 2> gpurun_out/n_tl.err || { echo "tl $v failed"; tail -5 gpurun_out/n_tl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/n_tl.json')); print('timelapse $v', round(d['value']), round(d['ms_per_step'],3), {k: round(x['us'],1) for k,x in d['kernels'].items()}, d['parity'])" | tee -a gpurun_out/n_summary.txt
done
