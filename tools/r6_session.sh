# Round-6 GPU session: tests, then the A/Bs of this round's switches (each step under its own limit, first failure ends it)
#   bash tools/r6_session.sh
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu.sh tests || exit 1
DVH_SCAN_SPAN=1 timeout -k 10 300 python -u -m pytest tests/test_vsg_gpu.py tests/test_synth10k_gpu.py tests/test_vsg_stack_more_gpu.py \
  tests/test_bench_job_gpu.py tests/test_workflow_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/span_tests.log 2>&1 \
  || { echo span tests failed; tail -20 gpurun_out/span_tests.log; exit 1; }
tail -1 gpurun_out/span_tests.log
bash tools/ab_env.sh span "DVH_SCAN_SPAN=0" "DVH_SCAN_SPAN=1" -- --steps 20 --warmup 3 || exit 1
bash tools/ab_env.sh wspan "DVH_SCAN_SPAN=0" "DVH_SCAN_SPAN=1" -- --workload weights --steps 20 --warmup 3 || exit 1
bash tools/ab_env.sh xq499 "DVH_VSTACK_XCDQ=1" "DVH_VSTACK_XCDQ=0" "DVH_SCAN_SPAN=1" -- --w499 --steps 20 --warmup 3 || exit 1
bash tools/ab_env.sh wxq499 "DVH_VSTACK_XCDQ=1" "DVH_VSTACK_XCDQ=0" -- --workload weights --w499 --steps 20 --warmup 3 || exit 1
bash tools/ab_env.sh sos "DVH_LIB=variants/sos_old.so" "DVH_LIB=das_diff_veh_amd/lib/libdvh.so" -- --workload prep --steps 20 --warmup 3 || exit 1
