# round-5: the reset draws the episode's demand into a table (imenv_draw_layout) for small launches:
# A/B against the in-kernel draw (IMENV_DTAB=0) on C5's shard and C4, then the GPU suite and smoke
set -o pipefail
O=${1:-gpurun_out/r5q}; mkdir -p $O
timeout -k 10 600 bash tools/ab_multi.sh $O/ab 3 "--config C2 --n-envs 131072|--config C4" \
  "dtab=IMENV_AB=1" "nodtab=IMENV_DTAB=0" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -3 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
