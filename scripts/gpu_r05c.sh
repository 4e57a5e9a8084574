# round-5 session c: product GPU suite (double-angle PE), then interleaved render and train timing
# against the per-frequency-sincos build (pe0)
set -u
cd "$GRAFT_REPO_ROOT"
L=loma-nerf_amd/lib
bash scripts/gpu_steps.sh tests || { echo "product tests failed"; exit 1; }
V="$L/libloma_nerf.so $L/libloma_nerf_pe0.so"
bash scripts/gpu_ab_render.sh $V $V && bash scripts/gpu_ab.sh $V $V $V
