# round-6 session n: in-process A/B at a fixed point (Adam lr 0: every build keeps the product's sane weights):
# the product, no floor guard (ng), k1 with half the LDS fragment reads (hl), k2 ablations abl1..5
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_ng.so $L/libloma_nerf_hl.so \
  $L/libloma_nerf_abl1.so $L/libloma_nerf_abl2.so $L/libloma_nerf_abl3.so $L/libloma_nerf_abl4.so \
  $L/libloma_nerf_abl5.so --lr 0 --rounds 24 --block 10 > gpurun_out/ab_n.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_n.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: v[m]['median'] for m in v})"; exit $rc
