# round-5: is the timed region's per-launch time at 131,072 envs inflated by the host enqueueing during
# execution? default / all K launches queued ahead (a 700 us lead) / device-memory kernel arguments
set -o pipefail
O=${1:-gpurun_out/r5e}; mkdir -p $O
timeout -k 10 900 bash tools/ab_multi.sh $O/ab 3 "--config C2 --n-envs 131072 --steps 150 --warmup 30" \
  "default=IMENV_AB=1" "queued=IMENV_BENCH_LEAD_US=700" "devka=HIP_FORCE_DEV_KERNARG=1" "devka_queued=HIP_FORCE_DEV_KERNARG=1;IMENV_BENCH_LEAD_US=700" \
  > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
