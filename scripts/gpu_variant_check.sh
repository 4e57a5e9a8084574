# A candidate library variant on one box: its GPU suite (LNERF_LIB), then interleaved bench timing
# against the default library.
#   gpurun -- bash scripts/gpu_variant_check.sh libloma_nerf_X.so
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
V="$PWD/$L/$1"
LNERF_LIB=$V timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "not single_hip_runtime" > gpurun_out/variant_tests.log 2>&1
rc=$?; echo "variant tests rc=$rc"; tail -n 3 gpurun_out/variant_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh $L/libloma_nerf.so $L/$1 $L/libloma_nerf.so $L/$1
