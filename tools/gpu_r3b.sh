#!/bin/bash
# Round-3 batch B: GPU suite (store policies incl. write-through), store-policy size sweep, consumer
# probe, 2-rank self-launched rehearsal with the gather.
OUT=gpurun_out/r3b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for c in C2 C4 C3; do
  for n in 131072 262144 524288 1048576; do
    for pol in plain "default:0" "default:1000000000000"; do
      p=${pol%%:*}; lim=${pol#*:}; tag=$p; [ "$p" = default ] && tag=wt_st$([ $lim = 0 ] && echo 0 || echo 1)
      if [ "$p" = default ]; then export IMENV_WT_STATE_MAX_BYTES=$lim; else unset IMENV_WT_STATE_MAX_BYTES; fi
      timeout -k 10 120 python bench.py --config $c --n-envs $n --store $p --no-cpu-baseline --no-alt-store --no-graph --steps 90 --warmup 30 > $OUT/sw_${c}_${n}_$tag.json 2> $OUT/sw_${c}_${n}_$tag.err || { echo "sweep failed $c $n $tag"; exit 1; }
      python -c "import json; d=json.load(open('$OUT/sw_${c}_${n}_$tag.json')); r=d['roofline']; print('$c', $n, '$tag', d['value'], r['kernel_us'], r['frac'], r['kernel'][:40])"
    done
  done
done
unset IMENV_WT_STATE_MAX_BYTES
for cn in C2:1048576 C4:131072 C3:262144; do
  c=${cn%%:*}; n=${cn##*:}
  for p in plain default stream; do
    timeout -k 10 120 python tools/consumer_probe.py --config $c --n-envs $n --store $p > $OUT/consumer_${c}_$p.json 2> $OUT/consumer_${c}_$p.err || { echo "consumer probe failed"; exit 1; }
    cat $OUT/consumer_${c}_$p.json
  done
done
for cn in C4:131072:plain C4:131072:default C3:262144:default C2:1048576:default C2:1048576:plain; do
  IFS=: read c n p <<< "$cn"
  IMENV_STAMPS=1 IMENV_JIT_OPTS=-DIMENV_STAMPS=1 timeout -k 10 120 python tools/stamp_probe.py --config $c --n-envs $n --store $p > $OUT/stamps_${c}_${n}_$p.json 2> $OUT/stamps_${c}_${n}_$p.err || { echo "stamp probe failed"; tail -5 $OUT/stamps_${c}_${n}_$p.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/stamps_${c}_${n}_$p.json')); print('$c $n $p', json.dumps(d['launches'][-1]))"
done
timeout -k 10 200 python bench.py --gpus 2 --rehearse-one-gpu --gather --steps 20 --warmup 5 --no-cpu-baseline > $OUT/rehearse2_gather.json 2> $OUT/rehearse2_gather.err || { echo "rehearse gather failed"; tail -20 $OUT/rehearse2_gather.err; exit 1; }
tail -1 $OUT/rehearse2_gather.json
echo done
