# Instruction-cache counters of k_qhull (208 KB of code) and k_pair at C3
# (run on the GPU box from the repo root): bash scripts/r4q_icache.sh
set -e
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs"
LQRO_QSIDE=0 timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/ic1 -o run -- $B > $O/ic1.log 2>&1
LQRO_QSIDE=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH_LEVEL SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d $O/ic2 -o run -- $B > $O/ic2.log 2>&1
python3 scripts/pmc_any.py $O/r4q_icache.json $O/ic1 $O/ic2
echo icache done
