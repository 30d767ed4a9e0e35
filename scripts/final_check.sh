# A round's final GPU pass (GPU box, repo root): bash scripts/final_check.sh TAG [1|2]
# (part 1: suite, smoke, k_qhull's traffic; part 2: profiles, bench, two ranks)
# the GPU suite, smoke, the stamped profiles (k_pair traffic and SQ counters,
# the kernel trace, k_qhull's traffic) and the bench line that cites them,
# then a two-rank rehearsal of bench.py's multi-GPU path on this one card
# (gloo: both ranks share it; timings not meaningful).  Every step has its
# own time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
TAG=${1:-rX}
O=gpurun_out/$TAG
PART=${2:-1}
mkdir -p $O
if [ "$PART" = 1 ]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/qhull_pmc.sh $TAG > $O/qhull_pmc.log 2>&1 || { tail -20 $O/qhull_pmc.log; exit 1; }
tail -3 $O/qhull_pmc.log
echo part 1 done
exit 0
fi
bash scripts/gpu_profile.sh $TAG > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
cp gpurun_out/${TAG}_* $O/ 2>/dev/null || true
LQRO_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_2ranks_gloo.json 2> $O/bench_2ranks_gloo.err || { tail -20 $O/bench_2ranks_gloo.err; exit 1; }
tail -c 300 $O/bench_2ranks_gloo.json
echo final check done
