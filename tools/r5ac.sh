# round-5: hand-over of raw Philox words (the reading step inverts) vs of values vs off: parity, A/B
set -o pipefail
O=${1:-gpurun_out/r5ac}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_drawn_fuzz_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "philox or traffic or drawn or continue" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 900 bash tools/ab_multi.sh $O/ab 3 "--config C2 --n-envs 131072" \
  "raw=IMENV_AB=1" "values=IMENV_DTAB_RAW=0" "off=IMENV_DTAB=0" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 900 bash tools/ab_multi.sh $O/ab2 2 "--config C2 --n-envs 262144|--config C2" \
  "off=IMENV_AB=1" "raw=IMENV_DTAB=1" > $O/ab2.log 2>&1 || { tail -20 $O/ab2.log; exit 1; }
cat $O/ab2.log
