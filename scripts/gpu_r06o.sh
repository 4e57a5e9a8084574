# round-6 session o: k1 on two 16-sample groups per wave at one wave per SIMD (libloma_nerf_g2.so,
# LNERF_K16_G2=1) -- its native parity and edge numerics, then the in-process A/B against the product
# and the pre-refactor k1 (pre: the same kernel before the pass machinery took NG groups)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
LNERF_LIB=$PWD/$L/libloma_nerf_g2.so timeout -k 10 500 python -u -m pytest tests/test_gpu_native.py tests/test_gpu_edge.py \
  -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_g2.log 2>&1
rc=$?; tail -5 gpurun_out/tests_g2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_pre.so $L/libloma_nerf_g2.so \
  --rounds 24 --block 10 > gpurun_out/ab_o.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_o.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: v[m]['median'] for m in v})"; exit $rc
