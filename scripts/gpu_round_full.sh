# Round evidence: GPU tests, default bench (with CPU baseline), render bench, precision report,
# rocprofv3 kernel stats + FETCH/WRITE PMC passes (each step under its own time limit).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed" gpurun_out/t1.log | tail -2
timeout -k 10 300 python bench.py > gpurun_out/b1.log 2>&1 || exit 1
tail -1 gpurun_out/b1.log | cut -c1-600
timeout -k 10 300 python bench.py --render --steps 5 --warmup 2 > gpurun_out/b_render.log 2>&1 || exit 1
tail -1 gpurun_out/b_render.log | cut -c1-400
timeout -k 10 300 python scripts/precision_report.py > gpurun_out/prec.log 2>&1 || exit 1
tail -5 gpurun_out/prec.log
bash scripts/gpu_profile.sh
