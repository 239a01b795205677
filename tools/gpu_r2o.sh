# Round-2 GPU session O: rocprofv3 kernel stats of the sliding bench (merged launch) and its f-v chain.
set -o pipefail
mkdir -p gpurun_out/prof_sl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sl -o r2_sliding --output-format csv -- python bench.py --workload sliding --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_sl/bench.json 2> gpurun_out/prof_sl/bench.err; echo prof=$?
find gpurun_out/prof_sl -name '*kernel_trace.csv' -delete
python - <<'PY'
import csv, glob, json
f = glob.glob('gpurun_out/prof_sl/**/r2_sliding_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us', r['Percentage'][:5])
d = json.loads(open('gpurun_out/prof_sl/bench.json').read())
print(round(d['value']), round(d['ms_per_step'], 2), {k: round(v, 2) for k, v in d['step_breakdown_ms'].items()})
PY
