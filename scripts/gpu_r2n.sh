# kact knob A/B: ring depth 6/8, timing experiments (fixed weight address, no epilogue, no stores)
set -u
cd "$GRAFT_REPO_ROOT"
L=loma-nerf_amd/lib
bash scripts/gpu_ab.sh $L/libloma_nerf.so || exit 1
LNERF_KACT=1 bash scripts/gpu_ab.sh $L/libloma_nerf.so $L/libloma_nerf_kr6.so $L/libloma_nerf_kr8.so $L/libloma_nerf_kwfix.so $L/libloma_nerf_knoepi.so $L/libloma_nerf_knost.so $L/libloma_nerf.so
