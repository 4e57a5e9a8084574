# The k16 schedule-robustness check on one box:
#   1. the full GPU suite on the default library;
#   2. the parity tests on the same source built under LLVM's max-ilp machine scheduler
#      (lib/libloma_nerf_ilp.so, `make defvariant V=ilp VDEFS="-mllvm -amdgpu-sched-strategy=max-ilp"`);
#   3. for the record, the round-3 k16 (csrc/variants/lnerf_k16_r3.hip, asm fragment reads and
#      asm operand split) under max-ilp on the cfg2 parity test that failed in round 3 (its rc is
#      reported, not required);
#   4. interleaved A/B timing of the default, round-3 and max-ilp libraries.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=loma-nerf_amd/lib
[ "${SKIP_DEFAULT_TESTS:-0}" = 1 ] || bash scripts/gpu_steps.sh tests || exit $?
LNERF_LIB=$PWD/$L/libloma_nerf_ilp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py \
  tests/test_gpu_edge.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/ilp_tests.log 2>&1
rc=$?; echo "ilp tests rc=$rc"; tail -n 3 gpurun_out/ilp_tests.log
[ $rc -eq 0 ] || exit $rc
if false && [ -f $L/libloma_nerf_r3ilp.so ]; then
  LNERF_LIB=$PWD/$L/libloma_nerf_r3ilp.so timeout -k 10 120 python -u -m pytest tests/test_gpu_native.py \
    -m gpu -q -p no:cacheprovider --timeout 60 --timeout-method thread -k "cfg2_all_rays" \
    > gpurun_out/r3ilp_tests.log 2>&1
  rc=$?; echo "r3 k16 under max-ilp: cfg2 parity rc=$rc (round 3: failed)"; tail -n 3 gpurun_out/r3ilp_tests.log
  [ $rc -le 1 ] || exit $rc   # 1 = test failures (expected possible); anything else is trouble
fi
bash scripts/gpu_ab.sh $L/libloma_nerf.so $L/libloma_nerf_r3.so $L/libloma_nerf_ilp.so \
  $L/libloma_nerf.so $L/libloma_nerf_r3.so $L/libloma_nerf_ilp.so
# the config-5 render: kr (default) vs k16's bf16 forward, interleaved
for i in 1 2; do
  for v in "" "--render-k16"; do
    timeout -k 10 120 python bench.py --render --steps 5 --warmup 2 $v > gpurun_out/render_ab.log 2>&1 || { echo "render $v failed"; tail -5 gpurun_out/render_ab.log; exit 1; }
    python -c "import json;d=json.loads([l for l in open('gpurun_out/render_ab.log') if l.startswith('{')][-1]);r=d['roofline'];print('render ${v:-kr}', round(d['ms_per_step'],2), 'ms/frame', r['kernel'], 'kernel', round(r.get('avg_ms',0),2), 'ms frac', round(r['frac'],3))"
  done
done
