# Round-2 GPU session C: validated-stack tests + bench (complement scan).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_synth10k_gpu.py tests/test_vsg_gpu.py tests/test_bench_job_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c_tests.log 2>&1; rc=$?
echo tests=$rc; tail -15 gpurun_out/c_tests.log
[ $rc -eq 0 ] || exit 1
bash tools/ab_validated.sh
