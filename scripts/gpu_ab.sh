# A/B of in-tree library variants: bench.py per lib (LNERF_LIB), fused/dw kernel times
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in "$@"; do
  LNERF_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-render ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/ab.log; exit 1; }
  python - "$lib" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/ab.log") if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[1], d["mfma"][:6], "ms/step %.4f" % d["ms_per_step"], {k: round(v, 4) for k, v in d["kernels_ms"].items()})
PY
done
