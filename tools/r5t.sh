# round-5: drawn-demand table with the one-round-trip draw kernel: parity (table on / off), A/B, trace
set -o pipefail
O=${1:-gpurun_out/r5t}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "philox or traffic or sharding" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 600 bash tools/ab_multi.sh $O/ab 2 "--config C2 --n-envs 131072|--config C4" \
  "dtab=IMENV_AB=1" "nodtab=IMENV_DTAB=0" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
for f in $O/ab/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['roofline']['reset_us'])"; done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/C4 -o p --output-format csv -- python bench.py --config C4 --no-cpu-baseline --no-alt-store --no-alt-obs --no-graph --steps 60 --warmup 30 > $O/C4.json 2> $O/C4.err || exit 1
grep -i "draw\|reset\|step" $O/C4/p_kernel_stats.csv | cut -c1-200
