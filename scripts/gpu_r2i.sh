# bench A/B of kact variants (timing knobs give wrong results by design)
set -u
cd "$GRAFT_REPO_ROOT"
L=loma-nerf_amd/lib
V="$L/libloma_nerf.so $L/libloma_nerf_knw.so $L/libloma_nerf_kns.so $L/libloma_nerf_kwf.so $L/libloma_nerf_kw3.so"
bash scripts/gpu_ab.sh $V || exit 1
bash scripts/gpu_ab.sh $V
