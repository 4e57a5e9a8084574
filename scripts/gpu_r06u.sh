# round-6 session u: round over round in one process -- the round-6 product against the round-5 final
# library (commit e4b77df, built from that tree: libloma_nerf_r5.so), 40 interleaved rounds
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_r5.so \
  --rounds 40 --block 10 > gpurun_out/ab_u.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_u.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: (v[m]['median'], v[m].get('mean')) for m in v})"; exit $rc
