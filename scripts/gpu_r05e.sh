# round-5 session e: GPU suite, then kr variants: resident head (HEADRES) x in-wave compositing
# (WAVECOMP), product = both on, h0wc0 = neither (the previous product)
set -u
cd "$GRAFT_REPO_ROOT"
L=loma-nerf_amd/lib
bash scripts/gpu_steps.sh tests || { echo "product tests failed"; exit 1; }
V="$L/libloma_nerf.so $L/libloma_nerf_wc0.so $L/libloma_nerf_h0.so $L/libloma_nerf_h0wc0.so"
bash scripts/gpu_ab_render.sh $V $V
