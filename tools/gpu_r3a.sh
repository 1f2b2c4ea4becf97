set -o pipefail
OUT=gpurun_out/r3a
mkdir -p $OUT
export TMPDIR=/tmp
IMENV_JIT_OPTS="-DIMENV_WT_STORE=1 -DIMENV_WT_STATE=1" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $OUT/parity_wt.log 2>&1 || { echo parity_wt failed; tail -20 $OUT/parity_wt.log; exit 1; }
tail -2 $OUT/parity_wt.log
bash tools/ab_multi.sh $OUT/ab 3 "--config C4|--config C3|--config C2 --steps 90 --warmup 30" "base=IMENV_AB=0" "wt=IMENV_JIT_OPTS=-DIMENV_WT_STORE=1" "wtst=IMENV_JIT_OPTS=-DIMENV_WT_STORE=1 -DIMENV_WT_STATE=1" || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
timeout -k 10 200 python bench.py --gpus 2 --rehearse-one-gpu --steps 20 --warmup 5 --cpu-seconds 0.5 > $OUT/rehearse2.json 2> $OUT/rehearse2.err || exit 1
timeout -k 10 200 python bench.py --gpus 2 --rehearse-one-gpu --gather --steps 20 --warmup 5 --no-cpu-baseline > $OUT/rehearse2_gather.json 2> $OUT/rehearse2_gather.err || exit 1
echo done
