# round-6 session q: dW on 16-wave workgroups (libloma_nerf_w16.so, LNERF_DW16_WAVES=16: four waves per
# SIMD at 128 registers, 2 x 2 tile blocks) -- native + edge parity, then the in-process A/B against the product
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
LNERF_LIB=$PWD/$L/libloma_nerf_w16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_native.py tests/test_gpu_edge.py \
  -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_w16.log 2>&1
rc=$?; tail -3 gpurun_out/tests_w16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_w16.so \
  --rounds 24 --block 10 > gpurun_out/ab_q.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_q.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: v[m]['median'] for m in v})"; exit $rc
