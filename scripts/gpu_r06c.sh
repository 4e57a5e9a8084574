# round-6 session c: the exceptional-row build -- edge numerics (report), the whole GPU suite, a bench
# line, then the in-process A/B: this build vs the round-5 product (libloma_nerf_r5.so) vs this build
# with f32 activation slabs (libloma_nerf_a32.so, LNERF_A24=0)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py -m gpu -x -v -s -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/edge.log 2>&1
rc=$?; grep -E "PASS|FAIL|exceptional|layer [0-9]|Error|error" gpurun_out/edge.log | tail -40; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_steps.sh tests bench || exit $?
L=loma-nerf_amd/lib
timeout -k 10 500 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_r5.so $L/libloma_nerf_a32.so \
  --rounds 30 --block 20 > gpurun_out/ab_c.log 2>&1
rc=$?; tail -45 gpurun_out/ab_c.log; exit $rc
