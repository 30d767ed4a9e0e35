# A/B of the C3 step: liblqro.so against variant libraries (GPU box, repo root):
#   bash scripts/ab_lib.sh OUT_TAG variant.so [variant2.so ...]
# each library runs c3_step.py (10 steps) twice, interleaved
set -e
T=$1; shift
O=gpurun_out
mkdir -p $O
for r in 1 2; do
  for v in liblqro.so "$@"; do
    echo "== $v run $r" >> $O/${T}_ab.txt
    LQRO_LIB=$v timeout -k 10 120 python3 scripts/c3_step.py 10 >> $O/${T}_ab.txt 2>&1
  done
done
grep -E "^==|steady" $O/${T}_ab.txt
echo ab done
