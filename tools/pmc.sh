# PMC passes (one counter group per run, kernel trace only) for the bench's kernels plus the
# FETCH_SIZE / WRITE_SIZE calibration program; writes gpurun_out/pmc_<tag>/ and the summary
# profiles/<tag>_pmc_summary.json (per-dispatch averages, calibrated HBM traffic per kernel).
#     bash tools/pmc.sh r2 [workload]     (workload != synth10k -> profiles/<tag>_pmc_summary_<workload>.json)
# The bench's launch layout (passes per stack launch, launches per step, chunk) is recorded in the
# summary: bench.py uses counters only from a summary whose layout equals its own run's.
set -o pipefail
tag=${1:-r1}
wl=${2:-synth10k}
sfx=""; [ "$wl" = synth10k ] || sfx="_$wl"
bargs="--workload $wl"; [ "$wl" = w499 ] && bargs="--workload synth10k --w499"  # synth10k at w = 499
[ "$wl" = weights_w499 ] && bargs="--workload weights --w499"  # configs[1] at w = 499
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_$tag$sfx
[ -x tools/calib/fetch_calib ] || { echo "build tools/calib/fetch_calib first"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmc_$tag$sfx/c$i -o pmc --output-format csv -- ./tools/calib/fetch_calib > /dev/null 2> gpurun_out/pmc_$tag$sfx/c$i.err || { echo "calib pass $i failed"; exit 1; }
done
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp -d gpurun_out/pmc_$tag$sfx/p$i -o pmc --output-format csv -- python bench.py $bargs --steps 2 --warmup 1 --no-cpu-baseline --layout-out gpurun_out/pmc_$tag$sfx/layout.json > /dev/null 2> gpurun_out/pmc_$tag$sfx/p$i.err || { echo "pmc pass $i failed"; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc_$tag$sfx profiles/${tag}_pmc_summary$sfx.json
