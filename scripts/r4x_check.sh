# full GPU suite + k_dynw time/traffic at HEAD's library (GPU box, repo root)
set -e
T=$1
O=gpurun_out
mkdir -p $O/$T
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/$T/gpu_tests.log 2>&1
tail -1 $O/$T/gpu_tests.log
bash scripts/r4w_dyn.sh $T
