# DVFS check (MI355X_MICROARCH.md 'DVFS give-back' item 1): the same step on random vs all-zero
# weights, interleaved; a large gap means the kernels run at a power-limited clock.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
for z in "" "--zero-weights"; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-render --no-cfg2 $z > gpurun_out/dvfs.log 2>&1 || { echo "failed $z"; tail -3 gpurun_out/dvfs.log; exit 1; }
  python -c "import json;d=json.loads([l for l in open('gpurun_out/dvfs.log') if l.startswith('{')][-1]);k=d['kernels_ms'];print('${z:-random}', round(d['ms_per_step'],4), 'k1', round(k['fused'],4), 'k2', round(k['dw'],4))"
done
done
