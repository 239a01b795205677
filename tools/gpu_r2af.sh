# Round-2 GPU session AF: full-size time-lapse parity (MFMA vs VALU f-v over 512 images, oracle on six).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_timelapse_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/af_tests.log 2>&1; rc=$?
echo tests=$rc; grep -E "passed|failed|max rel|Error|assert" gpurun_out/af_tests.log | tail -8
