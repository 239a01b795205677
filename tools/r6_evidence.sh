# Round-6 evidence: the GPU suite (assertion failures reported, not fatal to the profiling that follows), then the
# PMC summaries of the stack workloads.   bash tools/r6_evidence.sh TAG
set -o pipefail
tag=${1:-r6}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; echo gpu_tests=$rc; tail -3 gpurun_out/${tag}_gpu_tests.log; grep FAILED gpurun_out/${tag}_gpu_tests.log | head
[ $rc -le 1 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
for wl in ${WLS:-synth10k weights w499 weights_w499 sliding}; do
  bash tools/gpu.sh pmc $tag $wl || exit 1
  rm -rf gpurun_out/pmc_${tag}*/  # the raw counter CSVs (the summaries are copied to gpurun_out/; <= 64 MiB comes back)
done
