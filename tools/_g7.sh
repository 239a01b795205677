# fv_mfma images per block (G) sweep: time + HBM traffic of the f-v kernel on the time-lapse batch
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for g in 0 4 8; do
  DVH_FV_MG=$g timeout -k 10 200 python tools/bench_timelapse.py --steps 20 > gpurun_out/tl_g$g.json 2> gpurun_out/tl_g$g.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/tl_g$g.json').read().strip().splitlines()[-1]); print('G=$g fv us', round(d['fv_kernel']['us'],1))"
  rm -rf gpurun_out/pmc_g$g; mkdir -p gpurun_out/pmc_g$g
  for grp in FETCH_SIZE WRITE_SIZE; do
    DVH_FV_MG=$g timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmc_g$g/$grp -o pmc --output-format csv -- python tools/bench_timelapse.py --steps 2 --warmup 1 > /dev/null 2> gpurun_out/pmc_g$g/$grp.err || { echo pmc failed; exit 1; }
  done
  python tools/pmc_summary.py gpurun_out/pmc_g$g gpurun_out/pmc_g$g/s.json > /dev/null && python -c "import json; d=json.load(open('gpurun_out/pmc_g$g/s.json'))['fv_mfma_kernel']; print('G=$g fetch x2', round(d['fetch_bytes_x2']/1e9,3), 'GB write', round(d['write_bytes']/1e9,3), 'GB')"
done
