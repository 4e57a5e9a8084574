# GPU tests + precision report + bench in both fp32-class precisions
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/t1.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/precision_report.py > gpurun_out/prec.log 2>&1; echo "prec rc=$?"; tail -14 gpurun_out/prec.log
bash scripts/gpu_ab.sh loma-nerf_amd/lib/libloma_nerf.so
BENCH_ARGS=--f16x3 bash scripts/gpu_ab.sh loma-nerf_amd/lib/libloma_nerf.so loma-nerf_amd/lib/libloma_nerf.so
