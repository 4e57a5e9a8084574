# Iteration loop for the fused kernels: GPU tests, bench (default kernel), optional phase profile.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_k16.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/t_k16.log | tail -8
[ $rc -eq 0 ] || exit $rc
for k in ${K16_AB:-1}; do
  LNERF_K16=$k timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_k16_$k.log 2>&1 || exit 1
  python - "$k" <<'PY'
import json, sys
k = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/b_k16_{k}.log") if l.startswith("{")][-1])
print("K16=" + k, round(d["ms_per_step"], 4), {a: round(b, 4) for a, b in d["kernels_ms"].items()}, round(d["value"] / 1e6, 2), "M/s")
PY
done
if [ -n "${PROF:-}" ]; then
  LNERF_LIB=loma-nerf_amd/lib/libloma_nerf_prof.so timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bprof.log 2>&1
  grep "LNERF_PROF k16" gpurun_out/bprof.log | tail -1
fi
exit 0
