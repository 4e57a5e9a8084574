# round-end check of the shipped tree: GPU tests, smoke, default bench (with CPU baseline)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/b1.log 2>&1 || { tail -5 gpurun_out/b1.log; exit 1; }
tail -1 gpurun_out/b1.log | cut -c1-400
