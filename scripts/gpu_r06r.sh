# round-6 session r: the forward epilogue interleaved into the last k-step (EPIL) -- parity of the
# one-group (epil) and two-group (g2e) builds, then the in-process A/B against the product and g2
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
for v in epil g2e; do
  LNERF_LIB=$PWD/$L/libloma_nerf_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_native.py tests/test_gpu_edge.py \
    -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_$v.log 2>&1
  rc=$?; tail -3 gpurun_out/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_epil.so $L/libloma_nerf_g2.so \
  $L/libloma_nerf_g2e.so --rounds 24 --block 10 > gpurun_out/ab_r.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_r.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: v[m]['median'] for m in v})"; exit $rc
