# GPU tests, kact phase profile, then bench A/B kact vs k16
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/t1.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if [ -f loma-nerf_amd/lib/libloma_nerf_kprof.so ]; then
  LNERF_LIB=loma-nerf_amd/lib/libloma_nerf_kprof.so timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/kprof.log 2>&1
  grep LNERF_PROF gpurun_out/kprof.log | tail -1
fi
bash scripts/gpu_ab.sh loma-nerf_amd/lib/libloma_nerf.so
LNERF_KACT=0 bash scripts/gpu_ab.sh loma-nerf_amd/lib/libloma_nerf.so
bash scripts/gpu_ab.sh loma-nerf_amd/lib/libloma_nerf.so
