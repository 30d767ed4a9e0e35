# SQ counters of k_qhull (Qhull-order bench, C3): two passes, each its own run
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-qpmc}
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-roofline-probe"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $O/p1 -o run -- $B > $O/p1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH --output-format csv -d $O/p2 -o run -- $B > $O/p2.log 2>&1
python3 - $O <<'P'
import csv, glob, sys, collections
O = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for p in ("p1", "p2"):
    for f in glob.glob(f"{O}/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_qhull" not in k or "big" in k:
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:24s} {v:16.0f}")
P
