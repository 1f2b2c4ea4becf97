# round-5 bundle: GPU suite, host-interference A/B at 131,072 envs, bench lines, PMC summaries of the
# round-5 kernels, the large-capacity campaign under a time budget
set -o pipefail
O=${1:-gpurun_out/r5f}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -le 1 ] || exit 1
timeout -k 10 600 bash tools/ab_multi.sh $O/ab 2 "--config C2 --n-envs 131072 --steps 150 --warmup 30" \
  "default=IMENV_AB=1" "queued=IMENV_BENCH_LEAD_US=700" "devka=HIP_FORCE_DEV_KERNARG=1" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
timeout -k 10 300 python bench.py --n-envs 131072 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_131072_driver.json 2> $O/bench_131072.err || exit 1
echo benches done
CONFIGS="C2:1048576 C2:1048576:o64 C2:131072 C4:131072 C3:262144" timeout -k 10 1000 bash tools/profile_configs.sh $O/pmc > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
tail -3 $O/pmc.log
timeout -k 10 300 python -u tools/fuzz_gpu_campaign.py --big --envs 8 --cases 400 --start 870000 --budget 240 > $O/campaign_big.log 2>&1 || { tail -5 $O/campaign_big.log; exit 1; }
tail -1 $O/campaign_big.log
echo all done
