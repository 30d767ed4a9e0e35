# k_prio's hot-pair heuristic (LQRO_HOT_T seconds, LQRO_HOT_R metres) against
# the C3 step time (GPU box, repo root): bash scripts/hot_sweep.sh TAG
set -e
T=$1
O=gpurun_out
mkdir -p $O
for tr in "3 3" "2 3" "3 2" "2 2" "1.5 2" "1 1.5" "4 4"; do
  set -- $tr
  echo "== T=$1 R=$2" >> $O/${T}_hot.txt
  LQRO_HOT_T=$1 LQRO_HOT_R=$2 timeout -k 10 120 python3 scripts/c3_step.py 5 >> $O/${T}_hot.txt 2>&1
done
echo hot done
