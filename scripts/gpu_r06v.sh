# round-6 session v: the round's final library (one reduction after the guard's gated re-run) -- GPU
# suite, bench line, compat, kernel trace + HBM PMC + SQ counters of training and of the config-5
# render, RCCL world-size-1 steps; then round over round in one process against the round-5 library
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu_steps.sh tests bench compat trace pmc sq rtrace rpmc rsq dist || exit $?
L=loma-nerf_amd/lib
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_r5.so \
  --rounds 40 --block 10 > gpurun_out/ab_v.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_v.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: (v[m]['median'], v[m].get('mean')) for m in v})"; exit $rc
