# k_qhull's HBM traffic per build (stamped, for bench.py's `critical`) and its
# L2 hit rate (GPU box, repo root):  bash scripts/qhull_pmc.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-rX}
O=gpurun_out
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/qt_f -o run -- python3 scripts/qhull_traffic.py run $O/qt_run_f.json > $O/qt_f.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/qt_w -o run -- python3 scripts/qhull_traffic.py run $O/qt_run_w.json > $O/qt_w.log 2>&1
python3 scripts/qhull_traffic.py summarise $O/qt_f $O/qt_w $O/qt_run_f.json $O/${TAG}_qhull_traffic.json > /dev/null
cp $O/${TAG}_qhull_traffic.json profiles/${TAG}_qhull_traffic.json
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/qt_h -o run -- python3 scripts/qhull_traffic.py run $O/qt_run_h.json > $O/qt_h.log 2>&1
python3 scripts/pmc_any.py $O/${TAG}_qhull_l2.json $O/qt_h > $O/${TAG}_qhull_l2.txt 2>&1 || true
cat $O/${TAG}_qhull_l2.txt
echo qhull pmc done
