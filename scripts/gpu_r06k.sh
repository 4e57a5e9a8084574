# round-6 session k: dW workgroups of 16 waves (four per SIMD, 128 registers, 2 x 2 tile blocks;
# libloma_nerf_w16.so three half-blocks deep, _w16d2 two) -- fused/edge parity of each, then the
# in-process A/B against the product (8 waves, product-major MFMA order)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
for v in w16d2 w16; do
  LNERF_LIB=$PWD/$L/libloma_nerf_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_native.py tests/test_gpu_edge.py \
    -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_$v.log 2>&1
  rc=$?; tail -3 gpurun_out/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_w16.so $L/libloma_nerf_w16d2.so \
  --rounds 30 --block 20 > gpurun_out/ab_k.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_k.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: v[m]['median'] for m in v})"; exit $rc
