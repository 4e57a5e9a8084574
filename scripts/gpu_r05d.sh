# round-5 session d: kr scheduling barrier / read-ahead A/B (render), product render tests first
set -u
cd "$GRAFT_REPO_ROOT"
L=loma-nerf_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/tests_render.log 2>&1 || { tail -20 gpurun_out/tests_render.log; exit 1; }
tail -2 gpurun_out/tests_render.log
V="$L/libloma_nerf.so $L/libloma_nerf_s0.so $L/libloma_nerf_d3.so $L/libloma_nerf_d4.so"
bash scripts/gpu_ab_render.sh $V $V
