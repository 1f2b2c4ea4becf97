# round-5: the driver's short window without per-launch events: blocking vs polling end-of-window wait
set -o pipefail
O=${1:-gpurun_out/r5h}; mkdir -p $O
timeout -k 10 300 python tools/window_probe.py --no-events --rounds 20 > $O/window_131072.log 2>&1 || { tail -5 $O/window_131072.log; exit 1; }
ROC_ACTIVE_WAIT_TIMEOUT=1000 timeout -k 10 300 python tools/window_probe.py --no-events --rounds 20 > $O/window_131072_activewait.log 2>&1 || { tail -5 $O/window_131072_activewait.log; exit 1; }
timeout -k 10 300 python tools/window_probe.py --no-events --n-envs 1048576 --rounds 10 > $O/window_2p20.log 2>&1 || { tail -5 $O/window_2p20.log; exit 1; }
grep -h '^{"[a-z_0-9]*": {' $O/*.log | cut -c1-200
echo all done
