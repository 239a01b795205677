# Round-2 GPU session G: the new parity tests first, then the whole -m gpu suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_prep_gpu.py tests/test_vsg_stack_more_gpu.py tests/test_sliding_gpu.py -x -q --timeout 300 --timeout-method thread --durations=5 > gpurun_out/g_new.log 2>&1; rc=$?
echo new=$rc; tail -12 gpurun_out/g_new.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g_tests.log 2>&1; rc=$?
echo tests=$rc; tail -5 gpurun_out/g_tests.log
[ $rc -eq 0 ] || exit 1
