# A round's GPU check (run on the GPU box from the repo root):
#   bash scripts/round_check.sh TAG [pytest selection...]
# the GPU suite (or the given tests), smoke, a bench line.  Every step has its
# own time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
TAG=${1:-rX}
shift || true
O=gpurun_out/$TAG
mkdir -p $O
SEL=${@:-tests/}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $SEL > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['ms_per_step'],d['value']/1e6,json.dumps(d['critical']),json.dumps({k:(v['ms_per_step'],v.get('rank_shard_g8')) for k,v in d['configs'].items()}))"
echo done
