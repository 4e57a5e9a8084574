# round-6 session w: k1 reading weight fragments three tiles ahead (kd3, LNERF_K16_KDIST=3) on the NG-refactored
# pass machinery -- native parity, then the in-process A/B against the product
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
LNERF_LIB=$PWD/$L/libloma_nerf_kd3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_native.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_kd3.log 2>&1
rc=$?; tail -2 gpurun_out/tests_kd3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_kd3.so \
  --rounds 30 --block 10 > gpurun_out/ab_w.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_w.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: v[m]['median'] for m in v})"; exit $rc
