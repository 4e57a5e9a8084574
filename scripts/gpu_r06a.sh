# round-6 session a: product GPU suite, bench line, compat boundary re-timing, then the in-process
# A/B of f32 activation slabs (LNERF_A24=0, libloma_nerf_a32.so) against the int24 product
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu_steps.sh tests bench compat || exit $?
timeout -k 10 400 python scripts/ab_inproc.py loma-nerf_amd/lib/libloma_nerf.so loma-nerf_amd/lib/libloma_nerf_a32.so \
  --rounds 30 --block 20 > gpurun_out/ab_a32.log 2>&1
rc=$?; tail -40 gpurun_out/ab_a32.log; exit $rc
