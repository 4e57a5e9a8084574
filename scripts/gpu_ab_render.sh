# A/B of in-tree library variants on the config-5 render: bench.py --render per lib (LNERF_LIB),
# ms per frame and the render kernel's HIP-event time
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in "$@"; do
  LNERF_LIB=$lib timeout -k 10 120 python bench.py --render --steps 6 --warmup 2 > gpurun_out/abr.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/abr.log; exit 1; }
  python - "$lib" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/abr.log") if l.startswith("{")][-1]
d = json.loads(line)
r = d["roofline"]
print(sys.argv[1], "ms/frame %.3f" % d["ms_per_step"], "kernel %.3f" % r.get("avg_ms", 0), "kernel_frac %.3f" % r.get("kernel_frac", 0))
PY
done
