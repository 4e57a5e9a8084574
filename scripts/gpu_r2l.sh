# GPU tests (incl. opt-in kact parity), then bench default (k16) and kact
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|error|assert" gpurun_out/t1.log | head -20
[ $rc -eq 0 ] || exit $rc
L=loma-nerf_amd/lib
bash scripts/gpu_ab.sh $L/libloma_nerf.so || exit 1
LNERF_KACT=1 bash scripts/gpu_ab.sh $L/libloma_nerf.so || exit 1
