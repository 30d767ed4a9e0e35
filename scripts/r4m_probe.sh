set -e
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
LQRO_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-configs > $O/bench2.json 2> $O/bench2.err || { tail -20 $O/bench2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['rows_auto'], d['config']['parallelism'], str(d.get('host_cpp'))[:200])"
echo done
