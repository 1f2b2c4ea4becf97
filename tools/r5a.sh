# round-5 check: launch probes, the GPU suite with state records (default) and with rows only
# (IMENV_REC=0), int32 backlog_to rows, bench lines (driver form, C2 at 131,072, C4), RCCL graph gather
set -o pipefail
O=${1:-gpurun_out/r5a}; mkdir -p $O
timeout -k 10 240 python tools/probe_launch.py > $O/pl_default.json 2> $O/pl_default.err || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python tools/probe_launch.py > $O/pl_k1.json 2> $O/pl_k1.err || exit 1
echo probes done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -le 1 ] || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --n-envs 131072 --steps 150 --warmup 30 --no-cpu-baseline --no-alt-obs > $O/bench_131072_$i.json 2> $O/bench_131072_$i.err || exit 1
  IMENV_REC=0 timeout -k 10 300 python bench.py --n-envs 131072 --steps 150 --warmup 30 --no-cpu-baseline --no-alt-obs > $O/bench_131072_rows_$i.json 2> $O/bench_131072_rows_$i.err || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
timeout -k 10 300 python bench.py --config C4 --steps 150 --warmup 30 --no-cpu-baseline > $O/bench_C4.json 2> $O/bench_C4.err || exit 1
timeout -k 10 300 python bench.py --rccl-solo --n-envs 131072 --steps 60 --warmup 10 --no-cpu-baseline > $O/rccl_131072.json 2> $O/rccl_131072.err || exit 1
echo benches done
IMENV_REC=0 timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu_rows.log 2>&1; rc=$?
tail -3 $O/pytest_gpu_rows.log
[ $rc -le 1 ] || exit 1
IMENV_BTO_BYTES=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fuzz_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_bto32.log 2>&1; rc2=$?
tail -2 $O/pytest_bto32.log
[ $rc2 -le 1 ] || exit 1
echo all done
