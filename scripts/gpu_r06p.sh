# round-6 session p: the round's final library -- GPU suite, bench line, compat boundary re-timing,
# kernel trace + HBM PMC + SQ counters of training and of the config-5 render, the RCCL world-size-1
# steps, and the SQ counters of the two-group k1 (libloma_nerf_g2.so) for DESIGN's A/B entry
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu_steps.sh tests bench compat trace pmc sq rtrace rpmc rsq dist || exit $?
LNERF_LIB=$PWD/loma-nerf_amd/lib/libloma_nerf_g2.so bash scripts/gpu_sq.sh "$PWD/gpurun_out/sq_g2" \
  --steps 3 --warmup 1 --no-cpu-baseline --no-render --no-cfg2
