# round-5: drawn-demand fuzz (table forced on / default) and C4's state layout A/B (records vs rows)
set -o pipefail
O=${1:-gpurun_out/r5aa}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_drawn_fuzz_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/drawn_fuzz.log 2>&1 || { tail -40 $O/drawn_fuzz.log; exit 1; }
tail -2 $O/drawn_fuzz.log
timeout -k 10 600 bash tools/ab_multi.sh $O/ab 3 "--config C4" "rec=IMENV_AB=1" "rows=IMENV_REC=0" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
