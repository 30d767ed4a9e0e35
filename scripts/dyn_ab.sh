# k_dynw A/B (GPU box, repo root): bash scripts/dyn_ab.sh TAG variant.so [...]
# the GPU dynamics tests, then per library the kernel trace of dyn_prof.py
# (k_dynw's average duration) and its phase profile
set -e
export TMPDIR=/tmp
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dyn.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in liblqro.so "$@"; do
  LQRO_LIB=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 scripts/dyn_prof.py > $O/kt_$v.log 2>&1
  f=$(find $O/kt_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"; grep -i "k_dynw" $f | cut -d, -f1-8
  LQRO_LIB=$v LQRO_DYN_PROFILE=1 timeout -k 10 120 python3 scripts/dyn_prof.py > $O/prof_$v.txt 2>&1
  head -4 $O/prof_$v.txt
done
echo dyn ab done
