# Quick GPU check of a kernel change: GPU tests, then the default bench (no CPU baseline) twice.
#     bash tools/quick_ab.sh [extra bench args]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/qa_tests.log 2>&1; rc=$?
echo gpu_tests=$rc; tail -2 gpurun_out/qa_tests.log
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 "$@" > gpurun_out/qa_bench_$r.json 2> gpurun_out/qa_bench_$r.err || { tail -5 gpurun_out/qa_bench_$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/qa_bench_$r.json')); r=d['roofline']; print('value %.0f ms/step %.3f stack %.3f ms frac %.3f' % (d['value'], d['ms_per_step'], r['launch_ms'], r['frac']))"
done
