#!/bin/bash
# Round-3 C4 diagnosis of the current kernel at its BASELINE size (131,072 envs): ablations of each
# compute part (IMENV_ABLATE bits: 1 split, 2 demand draw, 4 observation values, 8 profit, 16 decode),
# the wave-count probe (65,536 envs = 1 wave per SIMD; 262,144 = 4), priority stagger, phase stamps.
OUT=${1:-gpurun_out/r3f}
export TMPDIR=/tmp
mkdir -p $OUT
B="python bench.py --config C4 --no-cpu-baseline --no-alt-store --no-graph --steps 90 --warmup 30"
show() { python -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['config']['n_envs_per_gpu'], r['kernel_us'], r['frac'])"; }
for r in 1 2; do
  for a in 0 1 2 4 8 16 31; do
    IMENV_JIT_OPTS="-DIMENV_ABLATE=$a" timeout -k 10 120 $B > $OUT/abl_${a}_$r.json 2> $OUT/abl_${a}_$r.err || { echo "ablation failed $a"; exit 1; }
    show $OUT/abl_${a}_$r.json "ablate=$a"
  done
  for n in 65536 262144; do
    timeout -k 10 120 $B --n-envs $n > $OUT/n${n}_$r.json 2> $OUT/n${n}_$r.err || { echo "size $n failed"; exit 1; }
    show $OUT/n${n}_$r.json "n=$n"
  done
  for pr in 1 3; do
    IMENV_JIT_OPTS="-DIMENV_PRIO=$pr" timeout -k 10 120 $B > $OUT/prio${pr}_$r.json 2> $OUT/prio${pr}_$r.err || { echo "prio failed"; exit 1; }
    show $OUT/prio${pr}_$r.json "prio=$pr"
  done
done
IMENV_STAMPS=1 IMENV_JIT_OPTS=-DIMENV_STAMPS=1 timeout -k 10 120 python tools/stamp_probe.py --config C4 > $OUT/stamps_C4.json 2> $OUT/stamps_C4.err || { echo "stamps failed"; exit 1; }
python -c "import json; d=json.load(open('$OUT/stamps_C4.json')); print(json.dumps(d['launches'][-1]))"
echo "r3f done"
