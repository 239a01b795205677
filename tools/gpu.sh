# The one GPU-session runner (run on the box through gpurun; every GPU step under its own time limit,
# steps chained so that the first failure ends the session).
#
#   bash tools/gpu.sh tests [pytest -k expr]     GPU test suite (-m gpu), then smoke()
#   bash tools/gpu.sh bench [bench args]         bench.py twice, no CPU baseline: value, step, stack launch
#   bash tools/gpu.sh ab LIB1 LIB2 ... [-- bench args]
#                                                A/B of variant libraries (python -m das_diff_veh_amd.build
#                                                variants/X.so DEF=1): vsg GPU tests, then the bench, per lib
#   bash tools/gpu.sh prof TAG [workload]        rocprofv3 --kernel-trace --stats of the bench ->
#                                                gpurun_out/prof_TAG*/ (copy the stats CSV to profiles/)
#   bash tools/gpu.sh pmc TAG [workload]         PMC passes -> profiles/TAG_pmc_summary[_workload].json
#   bash tools/gpu.sh final TAG                  end of round, first call: tests + smoke, PMC (synth10k, sliding,
#                                                weights, w = 499, timelapse); the second call is `lines`
#   bash tools/gpu.sh lines TAG [a|b]            every bench line with its CPU baseline (synth10k, weights, sliding,
#                                                timelapse, w = 499, prep, bootstrap, speeds-host) + kernel stats
set -o pipefail
mode=${1:-tests}; shift
mkdir -p gpurun_out
prof_env() { cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; }

run_tests() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" \
    > gpurun_out/gpu_tests.log 2>&1; local rc=$?
  echo gpu_tests=$rc; tail -3 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || return 1
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { echo smoke failed; tail -5 gpurun_out/smoke.log; return 1; }
  tail -1 gpurun_out/smoke.log
}

bench_line() {  # out-file, bench args...
  local out=$1; shift
  timeout -k 10 600 python bench.py "$@" > "$out" 2> "${out%.json}.err" || { tail -5 "${out%.json}.err"; return 1; }
  python - "$out" << 'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d.get("roofline") or {}
print("value %.0f %s  ms/step %.3f  launch %.3f ms  frac %.3f  traffic %s" % (
    d["value"], d["unit"], d["ms_per_step"], r.get("launch_ms", 0), r.get("frac", 0), r.get("traffic")))
PY
}

case $mode in
  tests)
    run_tests ${1:+-k "$1"} ;;
  bench)
    for r in 1 2; do bench_line gpurun_out/bench_$r.json --no-cpu-baseline --steps 40 "$@" || exit 1; done ;;
  ab)
    libs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done; [ "$1" = "--" ] && shift
    for v in "${libs[@]}"; do
      DVH_LIB=variants/$v.so timeout -k 10 300 python -m pytest tests/test_vsg_gpu.py tests/test_synth10k_gpu.py \
        -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/ab_tests_$v.log 2>&1; rc=$?
      echo tests_$v=$rc; tail -1 gpurun_out/ab_tests_$v.log; [ $rc -eq 0 ] || exit 1
    done
    for v in "${libs[@]}"; do
      echo -n "$v: "; DVH_LIB=variants/$v.so bench_line gpurun_out/ab_$v.json --no-cpu-baseline --steps 20 --warmup 3 "$@" \
        || exit 1
    done ;;
  prof)
    tag=$1; wl=${2:-synth10k}; sfx=""; [ "$wl" = synth10k ] || sfx="_$wl"
    prof_env
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag$sfx -o $tag$sfx --output-format csv \
      -- python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$tag$sfx.json \
      2> gpurun_out/prof_$tag$sfx.err || { tail -5 gpurun_out/prof_$tag$sfx.err; exit 1; }
    find gpurun_out/prof_$tag$sfx -name '*kernel_trace.csv' -delete ;;
  pmc)
    bash tools/pmc.sh "$1" "${2:-synth10k}" > gpurun_out/pmc_$1.log 2>&1 || { echo pmc failed; tail -5 gpurun_out/pmc_$1.log; exit 1; }
    sfx=""; [ "${2:-synth10k}" = synth10k ] || sfx="_$2"
    cp profiles/$1_pmc_summary$sfx.json gpurun_out/ ;;
  final)
    tag=$1
    run_tests || exit 1
    for wl in synth10k sliding weights w499 weights_w499; do
      bash "$0" pmc $tag $wl || exit 1
    done
    for o in fused corr7 corr; do  # weights: the SQ breakdown of the launch, the correlation alone, the plain kernel
      EXP_ARGS="--workload weights" timeout -k 10 400 bash tools/pmc_exp.sh ${tag}w_$o $o > gpurun_out/pmcx_${tag}w_$o.log 2>&1 \
        || { echo pmcx $o failed; tail -3 gpurun_out/pmcx_${tag}w_$o.log; exit 1; }
    done
    bash tools/pmc_timelapse.sh $tag > gpurun_out/pmc_tl.log 2>&1 || { echo pmc tl failed; tail -5 gpurun_out/pmc_tl.log; exit 1; }
    rm -rf gpurun_out/pmc_${tag}* ;;
  lines)  # part a: the VSG bench lines; part b: the rest + kernel stats (each fits one gpurun call)
    tag=$1; part=${2:-ab}
    if [[ $part == *a* ]]; then
      bench_line gpurun_out/${tag}_bench.json || exit 1
      bench_line gpurun_out/${tag}_bench_weights.json --workload weights || exit 1
      bench_line gpurun_out/${tag}_bench_sliding.json --workload sliding --steps 4 --warmup 1 || exit 1
      bench_line gpurun_out/${tag}_bench_w499.json --w499 || exit 1
      bench_line gpurun_out/${tag}_bench_weights_w499.json --workload weights --w499 || exit 1
    fi
    if [[ $part == *b* ]]; then
      bench_line gpurun_out/${tag}_bench_timelapse.json --workload timelapse || exit 1
      bench_line gpurun_out/${tag}_bench_prep.json --workload prep --steps 20 --warmup 3 || exit 1
      bench_line gpurun_out/${tag}_bench_bootstrap.json --workload bootstrap --steps 5 --warmup 1 || exit 1
      bench_line gpurun_out/${tag}_bench_speeds_host.json --workload speeds-host --steps 3 --warmup 1 || exit 1
      for wl in synth10k weights sliding timelapse prep bootstrap; do bash "$0" prof $tag $wl || exit 1; done
      bash "$0" profw499 $tag || exit 1
    fi ;;
  profw499)
    tag=$1
    prof_env
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_w499 -o ${tag}_w499 --output-format csv \
      -- python bench.py --w499 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${tag}_w499.json \
      2> gpurun_out/prof_${tag}_w499.err || { tail -5 gpurun_out/prof_${tag}_w499.err; exit 1; }
    find gpurun_out/prof_${tag}_w499 -name '*kernel_trace.csv' -delete ;;
  *)
    echo "unknown mode $mode"; exit 2 ;;
esac
