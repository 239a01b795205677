# Round-6 GPU session 2: where the fused launch's time goes with the covered-span scan, and its A/Bs
set -o pipefail
mkdir -p gpurun_out
for wl in synth10k weights; do
  timeout -k 10 300 python tools/exp_stack.py --workload $wl --only fused,corr7,corr --reps 5 > gpurun_out/r6_exp_$wl.json \
    2> gpurun_out/r6_exp_$wl.err || { echo exp $wl failed; tail -5 gpurun_out/r6_exp_$wl.err; exit 1; }
  echo "$wl: $(cat gpurun_out/r6_exp_$wl.json)"
done
bash tools/ab_env.sh span11 "DVH_LIB=das_diff_veh_amd/lib/libdvh.so" "DVH_LIB=variants/span11.so" -- --steps 20 --warmup 3 || exit 1
bash tools/ab_env.sh wspan11 "DVH_LIB=das_diff_veh_amd/lib/libdvh.so" "DVH_LIB=variants/span11.so" -- --workload weights --steps 20 --warmup 3 || exit 1
bash tools/ab_env.sh span499 "DVH_SCAN_SPAN=1" "DVH_SCAN_SPAN=2" -- --w499 --steps 20 --warmup 3 || exit 1
bash tools/ab_env.sh wspan499 "DVH_SCAN_SPAN=1" "DVH_SCAN_SPAN=2" -- --workload weights --w499 --steps 20 --warmup 3 || exit 1
for v in sos_split6 sos_split7; do
  DVH_LIB=variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_prep_gpu.py tests/test_integration_gpu.py -m gpu -q -x \
    --timeout 120 --timeout-method thread > gpurun_out/r6_${v}_tests.log 2>&1 || { echo $v tests failed; tail -10 gpurun_out/r6_${v}_tests.log; exit 1; }
  tail -1 gpurun_out/r6_${v}_tests.log
done
bash tools/ab_env.sh sossplit "DVH_LIB=das_diff_veh_amd/lib/libdvh.so" "DVH_LIB=variants/sos_split6.so" "DVH_LIB=variants/sos_split7.so" \
  -- --workload prep --steps 20 --warmup 3 || exit 1
bash tools/pmc_cmd.sh r6_prep sosm -- python bench.py --workload prep --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r6_prep_pmc.log 2>&1 \
  || { echo prep pmc failed; tail -5 gpurun_out/r6_prep_pmc.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_boot_gpu.py -m gpu -q -s --timeout 200 --timeout-method thread \
  -k "bootstrap_disp or convergence or mixed" > gpurun_out/r6_boot_audit.log 2>&1 || { echo boot audit failed; tail -20 gpurun_out/r6_boot_audit.log; exit 1; }
grep -h "picks equal\|near-tie\|column" gpurun_out/r6_boot_audit.log | head -20
