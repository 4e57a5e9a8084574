# round-6 session j: dW workgroups of 4 waves (one per SIMD, 512 registers; libloma_nerf_w4.so) --
# its GPU suite, then the in-process A/B against the 8-wave product
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
LNERF_LIB=$PWD/$L/libloma_nerf_w4.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/tests_w4.log 2>&1
rc=$?; tail -5 gpurun_out/tests_w4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_w4.so $L/libloma_nerf_p8.so \
  --rounds 30 --block 20 > gpurun_out/ab_j.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_j.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: v[m]['median'] for m in v})"; exit $rc
