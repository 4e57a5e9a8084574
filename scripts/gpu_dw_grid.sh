set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
for g in 0 384 768 1024; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-render --no-cfg2 --dw-grid $g > gpurun_out/grid.log 2>&1 || { echo "grid $g failed"; tail -3 gpurun_out/grid.log; exit 1; }
  python -c "import json;d=json.loads([l for l in open('gpurun_out/grid.log') if l.startswith('{')][-1]);k=d['kernels_ms'];print('grid $g', round(d['ms_per_step'],4), 'dw', round(k['dw'],4), 'reduce', round(k['reduce'],4), 'fused', round(k['fused'],4))"
done
done
