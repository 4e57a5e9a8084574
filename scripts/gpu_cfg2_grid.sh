set -u
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for g in 32 64 128 256 512; do
  timeout -k 10 120 python bench.py --config cfg2 --dw-grid $g --steps 50 --warmup 10 --no-render --no-cpu-baseline --no-cfg2 > gpurun_out/c2.log 2>&1 || { tail -3 gpurun_out/c2.log; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/c2.log') if l.startswith('{')][-1]); print($g, round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()})"
done; done
