#!/bin/bash
# Counters for BASELINE's small single-GPU configs at their BASELINE.json sizes (C4 131,072 envs,
# C3 262,144 envs; or the configs / sizes given in $CONFIGS as "name:n_envs ..."): a bench line, a
# kernel trace with stats, and one rocprofv3 --pmc pass per counter group (--pmc only, no sys/runtime
# trace), summarised by tools/pmc_summary.py keyed by the bench line's kernel_info. A config written
# "name:n_envs:o64" summarises the bench line's float64-observation kernel (roofline.alt_obs_f64) instead.
OUT=${1:-gpurun_out/cfgprof}
CONFIGS=${CONFIGS:-"C4:131072 C3:262144"}
export TMPDIR=/tmp
mkdir -p $OUT
python tools/pmc_calib.py build || exit 1
run() { tag=$1; shift; timeout -k 10 180 rocprofv3 --pmc "$@" -d $GRAFT_REPO_ROOT/$D/$tag -o p --output-format csv -- $CMD > $D/$tag.log 2>&1; }
CMD="python tools/pmc_calib.py"; D=$OUT; run cal_fetch FETCH_SIZE && run cal_write WRITE_SIZE || exit 1
for cn in $CONFIGS; do
  IFS=: read -r c n o <<< "$cn"
  if [ "$o" = "o64" ]; then
    D=$OUT/${c}_${n}_o64; ALT="--alt-obs-f64"; OBSFLAG=""
  else
    D=$OUT/${c}_$n; ALT=""; OBSFLAG="--no-alt-obs"
  fi
  mkdir -p $D
  BENCH="python bench.py --config $c --n-envs $n --no-cpu-baseline --no-alt-store $OBSFLAG --no-graph --steps 60 --warmup 30"
  timeout -k 10 240 $BENCH > $D/bench.json 2> $D/bench.err || exit 1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/trace -o p --output-format csv -- $BENCH > $D/bench_trace.json 2> $D/trace.err || exit 1
  CMD=$BENCH
  run fetch FETCH_SIZE && run write WRITE_SIZE &&
  run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY &&
  run sq2 SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS &&
  run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit 1
  python tools/pmc_summary.py $D/summary.json $n $OUT/cal_fetch $OUT/cal_write $D/fetch $D/write $D/sq1 $D/sq2 $D/tcc --bench-log $D/fetch.log --trace $D/trace/p_kernel_stats.csv $ALT > $D/summary.log 2>&1 || exit 1
  echo "$c $n done"
done
echo "profile_configs done"
