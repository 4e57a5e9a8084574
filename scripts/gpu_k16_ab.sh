# k16 A/B on one box: the GPU suite on the default library, then interleaved bench timing of the
# given variant libraries (default first), twice.
#   gpurun -- bash scripts/gpu_k16_ab.sh lib/libloma_nerf_X.so ...
set -u
cd "$GRAFT_REPO_ROOT"
L=loma-nerf_amd/lib
[ "${SKIP_DEFAULT_TESTS:-0}" = 1 ] || bash scripts/gpu_steps.sh tests || exit $?
libs="$L/libloma_nerf.so"
for v in "$@"; do libs="$libs $L/$v"; done
bash scripts/gpu_ab.sh $libs $libs
