# round-6 session i: in-process A/B of the A-slab formats: int24 (product), fp16 planes rescaled in
# k2 (ap), fp16 planes rebuilt and re-split in k2 (ap2)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_ap.so $L/libloma_nerf_ap2.so \
  --rounds 24 --block 20 > gpurun_out/ab_i.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_i.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: v[m]['median'] for m in v})"; exit $rc
