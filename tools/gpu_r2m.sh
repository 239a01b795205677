# Round-2 GPU session M: the whole -m gpu suite on the default library, then A/B of variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/m_tests.log 2>&1; rc=$?
echo tests=$rc; tail -4 gpurun_out/m_tests.log
[ $rc -eq 0 ] || exit 1
VARIANTS="${VARIANTS:-default}" bash tools/gpu_r2l.sh
