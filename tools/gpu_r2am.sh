# Round-2 GPU session AM: LDS-staged trajectories in pass_geometry_kernel (parity + bench), then the
# complement-scan A/B of tools/gpu_r2al.sh.
set -o pipefail
mkdir -p gpurun_out/r2am
timeout -k 10 400 python -u -m pytest tests/test_plan_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2am/tests.log 2>&1; rc=$?
echo tests=$rc; tail -1 gpurun_out/r2am/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r2am/tests.log | head -8; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r2am/bench.json 2> gpurun_out/r2am/bench.err || { echo "bench failed"; tail -5 gpurun_out/r2am/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2am/bench.json')); print('synth10k', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['frac'],3), {k: round(v,3) for k,v in d['step_breakdown_ms'].items()})"
bash tools/gpu_r2al.sh
