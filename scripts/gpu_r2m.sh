# render + train A/B: staggered k16 (default) vs unstaggered (lib ns); kact phase counters
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
for lib in $L/libloma_nerf.so $L/libloma_nerf_ns.so $L/libloma_nerf.so $L/libloma_nerf_ns.so; do
  LNERF_LIB=$lib timeout -k 10 120 python bench.py --render --steps 5 --warmup 2 > gpurun_out/r.log 2>&1 || { echo "$lib render failed"; tail -5 gpurun_out/r.log; exit 1; }
  echo "$lib render $(tail -1 gpurun_out/r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), "ms/frame")')"
done
bash scripts/gpu_ab.sh $L/libloma_nerf.so $L/libloma_nerf_ns.so $L/libloma_nerf.so || exit 1
LNERF_KACT=1 LNERF_LIB=$L/libloma_nerf_kprof.so timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/kprof.log 2>&1 || exit 1
grep LNERF_PROF gpurun_out/kprof.log | tail -2
