# Round-2 GPU session A: new GPU tests (device tables, configs[2] parity, bench job vs oracle), the
# rest of the GPU suite, then the synth10k headline bench (with CPU baseline) and a weights bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_plan_gpu.py tests/test_synth10k_gpu.py tests/test_bench_job_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/new_tests.log 2>&1; rc=$?
echo new_tests=$rc; tail -15 gpurun_out/new_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/bench_synth10k.json 2> gpurun_out/bench_synth10k.err || { tail -20 gpurun_out/bench_synth10k.err; exit 1; }
cat gpurun_out/bench_synth10k.json
timeout -k 10 300 python bench.py --workload weights --no-cpu-baseline > gpurun_out/bench_weights.json 2> gpurun_out/bench_weights.err || { tail -20 gpurun_out/bench_weights.err; exit 1; }
cat gpurun_out/bench_weights.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo gpu_tests=$rc; tail -5 gpurun_out/gpu_tests.log
