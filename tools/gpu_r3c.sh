#!/bin/bash
# Round-3 batch C: where the small-batch compute goes (ablation builds, WRONG results, timing only),
# plus SQ counters of the default kernels at BASELINE sizes.
OUT=gpurun_out/r3c
mkdir -p $OUT
export TMPDIR=/tmp
for cn in C4:131072 C3:262144; do
  c=${cn%%:*}; n=${cn##*:}
  for r in 1 2; do
    for a in 0 1 2 4 8 16 31; do
      IMENV_JIT_OPTS="-DIMENV_ABLATE=$a" timeout -k 10 120 python bench.py --config $c --n-envs $n --no-cpu-baseline --no-alt-store --no-graph --steps 90 --warmup 30 > $OUT/abl_${c}_${a}_$r.json 2> $OUT/abl_${c}_${a}_$r.err || { echo "ablation failed $c $a"; tail -5 $OUT/abl_${c}_${a}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/abl_${c}_${a}_$r.json')); r=d['roofline']; print('$c', 'ablate=$a', d['value'], r['kernel_us'], r['frac'])"
    done
  done
  BENCH="python bench.py --config $c --n-envs $n --no-cpu-baseline --no-alt-store --no-graph --steps 60 --warmup 30"
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $GRAFT_REPO_ROOT/$OUT/sq1_$c -o p --output-format csv -- $BENCH > $OUT/sq1_$c.log 2>&1 || { echo "sq1 failed"; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_WR SQ_BUSY_CYCLES -d $GRAFT_REPO_ROOT/$OUT/sq2_$c -o p --output-format csv -- $BENCH > $OUT/sq2_$c.log 2>&1 || { echo "sq2 failed"; exit 1; }
done
python tools/pmc_summary.py $OUT/sq_summary.json 131072 $OUT/sq1_C4 $OUT/sq2_C4 > $OUT/sq_C4.log 2>&1
python tools/pmc_summary.py $OUT/sq_summary3.json 262144 $OUT/sq1_C3 $OUT/sq2_C3 > $OUT/sq_C3.log 2>&1
grep imenv_step $OUT/sq_C4.log $OUT/sq_C3.log
echo done
