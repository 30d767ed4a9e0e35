# k_qhull's instruction fetch: SQC instruction-cache requests, hits and misses
# per launch beside k_pair's (GPU box, repo root):  bash scripts/qhull_icache.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-rX}
O=gpurun_out
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $O/ic_a -o run -- python3 scripts/c3_step.py 3 > $O/ic_a.log 2>&1
python3 scripts/pmc_any.py $O/${TAG}_qhull_icache.json $O/ic_a > $O/${TAG}_qhull_icache.txt 2>&1 || true
cat $O/${TAG}_qhull_icache.txt
echo icache pmc done
