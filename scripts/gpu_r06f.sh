# round-6 session f: exceptional rows v3 (scan only in splits that met one) -- GPU suite, bench line,
# in-process A/B against the round-5 product and the no-xrow build
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py -m gpu -v -s -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/edge.log 2>&1
grep -E "FAIL|exceptional|tiny-sigma|rror" gpurun_out/edge.log | cut -c1-300 | tail -20
bash scripts/gpu_steps.sh tests bench || exit $?
L=loma-nerf_amd/lib
timeout -k 10 600 python scripts/ab_inproc.py $L/libloma_nerf.so $L/libloma_nerf_r5.so $L/libloma_nerf_nx.so \
  --rounds 30 --block 20 > gpurun_out/ab_f.log 2>&1
rc=$?; python3 -c "
import json; t=open('gpurun_out/ab_f.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(k, {m: v[m]['median'] for m in v})"; exit $rc
