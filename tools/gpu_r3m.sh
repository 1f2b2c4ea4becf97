#!/bin/bash
# Round-3: XCD-aware env chunks for small-block launches (IMENV_XCD_REMAP, default 1) vs identity,
# interleaved 4x for C4 at 131,072 and C2 at 131,072; a PMC FETCH/WRITE pass of C4 with each; then
# the whole GPU suite (its full-size C4 / C2 cases run the remapped grid).
OUT=${1:-gpurun_out/r3m}
export TMPDIR=/tmp
mkdir -p $OUT
show() { python -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; print('$2', d['config']['n_envs_per_gpu'], r['kernel_us'], r['frac'], json.dumps(r.get('launch_pacing')))"; }
B="python bench.py --no-cpu-baseline --no-alt-store --no-graph --steps 150 --warmup 30"
for r in 1 2 3 4; do
  for v in 1 0; do
    IMENV_JIT_OPTS="-DIMENV_XCD_REMAP=$v" timeout -k 10 120 $B --config C4 > $OUT/C4_x${v}_$r.json 2> $OUT/C4_x${v}_$r.err || { echo "bench failed"; exit 1; }
    show $OUT/C4_x${v}_$r.json "C4 remap=$v"
    IMENV_JIT_OPTS="-DIMENV_XCD_REMAP=$v" timeout -k 10 120 $B --config C2 --n-envs 131072 > $OUT/C2s_x${v}_$r.json 2> $OUT/C2s_x${v}_$r.err || { echo "bench failed"; exit 1; }
    show $OUT/C2s_x${v}_$r.json "C2s remap=$v"
  done
done
python tools/pmc_calib.py build || exit 1
for v in 1 0; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    IMENV_JIT_OPTS="-DIMENV_XCD_REMAP=$v" timeout -k 10 180 rocprofv3 --pmc $ctr -d $GRAFT_REPO_ROOT/$OUT/pmc_x${v}_$ctr -o p --output-format csv -- python bench.py --config C4 --no-cpu-baseline --no-alt-store --no-graph --steps 60 --warmup 30 > $OUT/pmc_x${v}_$ctr.log 2>&1 || { echo "pmc failed"; exit 1; }
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
echo "r3m done"
