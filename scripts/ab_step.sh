# A/B of the C3 step between liblqro.so and variant libraries (GPU box, repo root):
#   bash scripts/ab_step.sh OUT_TAG variant.so [variant2.so ...]
# each library runs c3_step.py twice, interleaved; then the Qhull-order parity
# tests on liblqro.so
set -e
T=$1; shift
O=gpurun_out
mkdir -p $O
for r in 1 2; do
  for v in liblqro.so "$@"; do
    echo "== $v run $r" >> $O/${T}_ab.txt
    LQRO_LIB=$v timeout -k 10 120 python3 scripts/c3_step.py 6 >> $O/${T}_ab.txt 2>&1
  done
done
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_qhull_order.py > $O/${T}_tests.txt 2>&1
tail -2 $O/${T}_tests.txt
echo ab done
