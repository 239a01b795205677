# Round-2 GPU session AP: the full GPU suite + smoke on the committed tree, then tools/gpu_r2ao.sh (the
# scales-overlap patch applied on the box).
set -o pipefail
mkdir -p gpurun_out/r2ap
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2ap/tests.log 2>&1; rc=$?
echo gpu_tests=$rc; tail -1 gpurun_out/r2ap/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r2ap/tests.log | head -8; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2ap/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/r2ap/smoke.log; exit 1; }
tail -1 gpurun_out/r2ap/smoke.log
bash tools/gpu_r2ao.sh
