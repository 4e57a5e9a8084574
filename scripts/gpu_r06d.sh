# round-6 session d: the deficit-only exceptional rows with pipelined gathers -- GPU suite, then the
# in-process A/B against the round-5 product (r5), this build without the exceptional-row pass (nx),
# and this build with f32 activation slabs (a32)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py -m gpu -x -v -s -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/edge.log 2>&1
rc=$?; grep -E "FAIL|exceptional|layer [0-9]|tiny-sigma|Error|error" gpurun_out/edge.log | tail -30; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_steps.sh tests || exit $?
L=loma-nerf_amd/lib
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_r5.so $L/libloma_nerf_nx.so $L/libloma_nerf_a32.so \
  --rounds 30 --block 20 > gpurun_out/ab_d.log 2>&1
rc=$?; tail -60 gpurun_out/ab_d.log | grep -v "^round"; exit $rc
