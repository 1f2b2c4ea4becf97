# round-5: the driver's short window at 131,072 envs (tools/window_probe.py), and records vs rows timed
# with a deep launch queue (IMENV_BENCH_LEAD_US: no host-paced gaps inside the event pairs)
set -o pipefail
O=${1:-gpurun_out/r5g}; mkdir -p $O
timeout -k 10 300 python tools/window_probe.py > $O/window_131072.log 2>&1 || { tail -5 $O/window_131072.log; exit 1; }
tail -1 $O/window_131072.log | cut -c1-300
timeout -k 10 300 python tools/window_probe.py --n-envs 1048576 --rounds 8 > $O/window_2p20.log 2>&1 || { tail -5 $O/window_2p20.log; exit 1; }
timeout -k 10 900 bash tools/ab_multi.sh $O/ab 3 "--config C2 --n-envs 131072 --steps 150 --warmup 30|--config C4 --steps 150 --warmup 30" \
  "rec=IMENV_BENCH_LEAD_US=700" "rows=IMENV_BENCH_LEAD_US=700;IMENV_REC=0" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
echo all done
