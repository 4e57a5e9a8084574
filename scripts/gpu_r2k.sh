# GPU tests, kact phase profile, then bench A/B of kact variants vs k16
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|error|assert" gpurun_out/t1.log | head -20
[ $rc -eq 0 ] || exit $rc
LNERF_LIB=loma-nerf_amd/lib/libloma_nerf_kprof.so timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/kprof.log 2>&1 || exit 1
grep LNERF_PROF gpurun_out/kprof.log | tail -1
L=loma-nerf_amd/lib
bash scripts/gpu_ab.sh $L/libloma_nerf.so $L/libloma_nerf_kpr.so || exit 1
LNERF_KACT=0 bash scripts/gpu_ab.sh $L/libloma_nerf.so || exit 1
bash scripts/gpu_ab.sh $L/libloma_nerf.so $L/libloma_nerf_kpr.so
LNERF_KACT=0 bash scripts/gpu_ab.sh $L/libloma_nerf.so || exit 1
