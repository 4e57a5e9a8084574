# round-6 session t: what the exceptional-row machinery costs k2 -- in-process A/B of the product against
# the same library without it (nx, LNERF_DW16_XROW=0: round 5's plain balanced split for every row)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_nx.so \
  --rounds 30 --block 10 > gpurun_out/ab_t.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_t.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: v[m]['median'] for m in v})"; exit $rc
