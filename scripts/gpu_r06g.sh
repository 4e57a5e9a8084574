# round-6 session g: A slabs as k1's fp16 planes (libloma_nerf_ap.so, LNERF_A16P=1) -- its GPU suite
# (native parity + edge numerics), then the in-process A/B against the int24 product
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
LNERF_LIB=$PWD/$L/libloma_nerf_ap.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/tests_ap.log 2>&1
rc=$?; tail -5 gpurun_out/tests_ap.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_ap.so \
  --rounds 30 --block 20 > gpurun_out/ab_g.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_g.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: v[m]['median'] for m in v})"; exit $rc
