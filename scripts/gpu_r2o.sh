# kact parity (new epilogue) then kact A/B new vs previous epilogue
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/t1.log | head -12
[ $rc -eq 0 ] || exit $rc
LNERF_KACT=1 bash scripts/gpu_ab.sh $L/libloma_nerf.so $L/libloma_nerf_kold.so $L/libloma_nerf.so $L/libloma_nerf_kold.so || exit 1
bash scripts/gpu_ab.sh $L/libloma_nerf.so || exit 1
