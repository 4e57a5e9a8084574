# round-5 session f: k1 variants SPREAD2 (DMA over both k-steps of a chunk), ONECHUNK (one-tile
# passes as one chunk), WAVECOMP (in-wave compositing scans): the combined variant's GPU suite,
# then interleaved timing
set -u
cd "$GRAFT_REPO_ROOT"
L=loma-nerf_amd/lib
LNERF_LIB=$PWD/$L/libloma_nerf_all3.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "not single_hip_runtime" > gpurun_out/variant_tests.log 2>&1
rc=$?; echo "all3 tests rc=$rc"; tail -n 3 gpurun_out/variant_tests.log
[ $rc -eq 0 ] || exit $rc
V="$L/libloma_nerf.so $L/libloma_nerf_sp2.so $L/libloma_nerf_hc.so $L/libloma_nerf_wc.so $L/libloma_nerf_all3.so"
bash scripts/gpu_ab.sh $V $V
