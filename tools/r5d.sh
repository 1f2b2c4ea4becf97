# round-5: slim JIT kernels (no info code, no tail guards) A/B at C5's shard and C4, then the GPU suite
set -o pipefail
O=${1:-gpurun_out/r5d}; mkdir -p $O
timeout -k 10 900 bash tools/ab_multi.sh $O/ab 3 "--config C2 --n-envs 131072 --steps 150 --warmup 30|--config C4 --steps 150 --warmup 30" \
  "slim_rec=IMENV_AB=1" "full_rec=IMENV_JIT_SLIM=0" "slim_rows=IMENV_REC=0" "full_rows=IMENV_REC=0;IMENV_JIT_SLIM=0" \
  > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 200 python tools/probe_launch.py > $O/pl.json 2> $O/pl.err || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -le 1 ] || exit 1
echo all done
