# Round-2 GPU session AI: guessed-start searches + 1024-thread blocks in pass_geometry_kernel -- geometry parity, then the headline bench.
set -o pipefail
mkdir -p gpurun_out/r2ai
timeout -k 10 400 python -u -m pytest tests/test_plan_gpu.py tests/test_vsg_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2ai/tests.log 2>&1; rc=$?
echo tests=$rc; tail -3 gpurun_out/r2ai/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r2ai/bench.json 2> gpurun_out/r2ai/bench.err || { echo "bench failed"; tail -5 gpurun_out/r2ai/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2ai/bench.json')); print('synth10k', round(d['value']), round(d['ms_per_step'],2), {k: round(v,3) for k,v in d['step_breakdown_ms'].items()})"
