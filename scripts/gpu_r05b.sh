# round-5 session b: product GPU suite, then interleaved timing of the k2 head-split variants and the
# k1 pin/FDSRC-off build against the product library
set -u
cd "$GRAFT_REPO_ROOT"
L=loma-nerf_amd/lib
bash scripts/gpu_steps.sh tests; echo "product tests rc=$?"
V="$L/libloma_nerf.so $L/libloma_nerf_hw1.so $L/libloma_nerf_hw3.so $L/libloma_nerf_hx0.so $L/libloma_nerf_pin0.so"
bash scripts/gpu_ab.sh $V $V
