# PMC passes (one group per run, kernel trace only) over tools/bench_timelapse.py:
# writes profiles/<tag>_pmc_summary_timelapse.json (copied to gpurun_out/).   bash tools/pmc_timelapse.sh TAG
set -o pipefail
tag=${1:-r1}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
d=gpurun_out/pmc_${tag}_timelapse
mkdir -p $d
[ -x tools/calib/fetch_calib ] || { echo "build tools/calib/fetch_calib first"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $d/c$i -o pmc --output-format csv -- ./tools/calib/fetch_calib > /dev/null 2> $d/c$i.err || { echo "calib pass $i failed"; exit 1; }
done
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $d/p$i -o pmc --output-format csv -- python tools/bench_timelapse.py --steps 2 --warmup 1 > /dev/null 2> $d/p$i.err || { echo "pmc pass $i failed"; tail -3 $d/p$i.err; exit 1; }
done
# MFMA activity (its own pass; a counter this rocprofv3 does not know only loses this pass)
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 -d $d/p9 -o pmc --output-format csv -- python tools/bench_timelapse.py --steps 2 --warmup 1 > /dev/null 2> $d/p9.err || { echo "mfma pass failed (kept going)"; tail -2 $d/p9.err; rm -rf $d/p9; }
python tools/pmc_summary.py $d profiles/${tag}_pmc_summary_timelapse.json && cp profiles/${tag}_pmc_summary_timelapse.json gpurun_out/
rm -rf $d
