#!/bin/bash
OUT=gpurun_out/prio
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/ab_multi.sh $OUT 3 "--config C4 --steps 90 --warmup 30|--config C3 --steps 90 --warmup 30|--config C2 --steps 60 --warmup 30" "p0=IMENV_AB=0" "p1=IMENV_JIT_OPTS=-DIMENV_PRIO=1" "p3=IMENV_JIT_OPTS=-DIMENV_PRIO=3"
