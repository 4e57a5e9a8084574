# dW workgroup budget re-sweep for dw16 fp16x3 (LNERF_DW_GRID, env only)
set -u
cd "$GRAFT_REPO_ROOT"
L=loma-nerf_amd/lib/libloma_nerf.so
for g in 512 768 1024 384 512 768 1024; do
  echo "LNERF_DW_GRID=$g"; LNERF_DW_GRID=$g bash scripts/gpu_ab.sh $L || exit 1
done
