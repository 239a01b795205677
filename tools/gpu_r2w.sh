# Round-2 GPU session W: MFMA f-v kernel time breakdown (experiment builds with parts removed; wrong results).
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/w_summary.txt
tl() {  # tag, then env assignments
  tag=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_timelapse.py --steps 5 > gpurun_out/w_tl.json 2> gpurun_out/w_tl.err || { echo "tl $tag failed"; tail -5 gpurun_out/w_tl.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/w_tl.json')); print('timelapse $tag', round(d['value']), round(d['ms_per_step'],3), {k: round(x['us'],1) for k,x in d['kernels'].items()})" | tee -a gpurun_out/w_summary.txt
}
V=das_diff_veh_amd/lib/variants
tl default A=1 && tl nostore DVH_LIB=$V/exp1.so && tl nosample DVH_LIB=$V/exp2.so && tl nomfma DVH_LIB=$V/exp3.so || exit 1
