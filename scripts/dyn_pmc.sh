# k_dynw SQ counters (GPU box, repo root): bash scripts/dyn_pmc.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-rX}
O=gpurun_out
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/dp_1 -o run -- python3 scripts/dyn_prof.py > $O/dp_1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VALU --output-format csv -d $O/dp_2 -o run -- python3 scripts/dyn_prof.py > $O/dp_2.log 2>&1 || true
python3 scripts/pmc_any.py $O/${TAG}_dyn_pmc.json $O/dp_1 $O/dp_2 > /dev/null
python3 - $O/${TAG}_dyn_pmc.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if "k_dynw" in k:
        w = v.get("SQ_WAVES", 1) or 1
        print(k, "launches", v["launches"])
        for c in sorted(v):
            if c != "launches":
                print(f"  {c:28s} {v[c]:16.0f}  per wave {v[c] / w:12.1f}")
PY
