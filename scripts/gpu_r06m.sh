# round-6 session m: the fp16x3 floor guard (head row + hidden rows) -- edge numerics, the whole GPU suite,
# a bench line; then the k2 bottleneck ablations (no MFMA / no split / no loads) and k1 with half the LDS
# fragment reads (hl), in-process against the product
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py -m gpu -v -s -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/edge.log 2>&1
rc=$?; grep -E "FAIL|guard|rror" gpurun_out/edge.log | cut -c1-300 | tail -30; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_steps.sh tests bench || exit $?
L=loma-nerf_amd/lib
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_abl1.so $L/libloma_nerf_abl2.so \
  $L/libloma_nerf_abl3.so $L/libloma_nerf_hl.so --rounds 16 --block 10 > gpurun_out/ab_m.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_m.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: v[m]['median'] for m in v})"; exit $rc
