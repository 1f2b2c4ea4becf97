# round-5: the one-period-ahead hand-over (every step draws period t+1 off its chain) vs the four-period
# one vs none: parity with the ahead form forced, then A/B on C5's shard, C4 and C3
set -o pipefail
O=${1:-gpurun_out/r5ap}; mkdir -p $O
IMENV_DTAB_AHEAD=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_drawn_fuzz_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "philox or drawn or continue" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 1200 bash tools/ab_multi.sh $O/ab 3 "--config C2 --n-envs 131072|--config C4|--config C3" \
  "block=IMENV_AB=1" "ahead=IMENV_DTAB_AHEAD=1;IMENV_DTAB=1" "off=IMENV_DTAB=0" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
