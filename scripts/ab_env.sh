# A/B of the C3 step across environment settings (GPU box, repo root):
#   bash scripts/ab_env.sh OUT_TAG "ENV=..." ["ENV=..." ...]   ("-": the defaults)
# each setting runs c3_step.py twice, interleaved
set -e
T=$1; shift
O=gpurun_out
mkdir -p $O
for r in 1 2; do
  for v in "$@"; do
    echo "== $v run $r" >> $O/${T}_ab.txt
    if [ "$v" = "-" ]; then
      timeout -k 10 120 python3 scripts/c3_step.py 10 >> $O/${T}_ab.txt 2>&1
    else
      env $v timeout -k 10 120 python3 scripts/c3_step.py 10 >> $O/${T}_ab.txt 2>&1
    fi
  done
done
grep -E "^==|steady" $O/${T}_ab.txt
echo ab done
