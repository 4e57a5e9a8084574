# round-5 session g: the non-default modes of the final library, labelled lines
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for a in "--x6-train" "--input points" "--no-optimizer" "--render --x6"; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-cfg2 --no-render $a > gpurun_out/v.log 2>&1 || { echo "$a failed"; tail -3 gpurun_out/v.log; exit 1; }
  python -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/v.log') if l.startswith('{')][-1])
print('$a', round(d['ms_per_step'],4), d.get('dtype'), round(d['roofline']['frac'],3), d['config'].get('variant'))"
done
