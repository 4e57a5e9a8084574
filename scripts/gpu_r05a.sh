# round-5 A/B session: product GPU suite, cfg3-size parity of the staggered k1 variants, then
# interleaved timing of the k1 / k2 / kr variants (one box, each step under its own limit)
set -u
cd "$GRAFT_REPO_ROOT"
L=loma-nerf_amd/lib
bash scripts/gpu_steps.sh tests; echo "product tests rc=$?"
for v in s2 s2p; do
  LNERF_LIB=$PWD/$L/libloma_nerf_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "full_size" > gpurun_out/var_$v.log 2>&1
  rc=$?; echo "variant $v parity rc=$rc: $(tail -1 gpurun_out/var_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
V="$L/libloma_nerf_base.so $L/libloma_nerf_p2f.so $L/libloma_nerf_s2.so $L/libloma_nerf_s2p.so $L/libloma_nerf.so $L/libloma_nerf_o1.so $L/libloma_nerf_hx0.so"
bash scripts/gpu_ab.sh $V $V || exit $?
bash scripts/gpu_ab_render.sh $L/libloma_nerf.so $L/libloma_nerf_ks.so $L/libloma_nerf.so $L/libloma_nerf_ks.so
