set -e
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python scripts/crowded.py --qhull 40.3 30 22 > $O/r3g_crowded_qhull.txt 2>&1
LQRO_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/r3g_bench2_gloo.json 2> $O/r3g_bench2_gloo.err
echo done
