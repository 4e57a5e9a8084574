# SQ PMC of kact: product vs the no-epilogue timing variant
set -u
cd "$GRAFT_REPO_ROOT"
echo "== product"; bash scripts/gpu_pmc_sq3.sh || exit 1
echo "== kne"; LNERF_LIB=$GRAFT_REPO_ROOT/loma-nerf_amd/lib/libloma_nerf_kne.so bash scripts/gpu_pmc_sq3.sh || exit 1
