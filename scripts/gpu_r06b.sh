# round-6 session b: the exceptional-row build -- edge numerics first, then the whole GPU suite and a
# bench line (each step under its own limit, stopping at the first failure)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py -m gpu -x -v -s -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/edge.log 2>&1
rc=$?; grep -E "PASS|FAIL|exceptional|Error|error" gpurun_out/edge.log | tail -30; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_steps.sh tests bench
