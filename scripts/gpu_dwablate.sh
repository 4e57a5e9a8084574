set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for m in 0 1 2; do
  LNERF_DW_MODE=$m timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/abl_$m.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/abl_$m.log').read().strip().splitlines()[-1]); print('mode $m', d['kernels_ms'])"
done
