# round-6 session l: the fp16x3 floor guard -- edge numerics (report), the whole GPU suite, a bench line
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py -m gpu -v -s -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/edge.log 2>&1
rc=$?; grep -E "FAIL|PASS|guard|exceptional|rror" gpurun_out/edge.log | cut -c1-300 | tail -30; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_steps.sh tests bench
