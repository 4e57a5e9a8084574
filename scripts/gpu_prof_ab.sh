# phase counters (LNERF_PROF builds) of in-tree library variants
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in "$@"; do
  LNERF_LIB=$lib timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pab.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/pab.log; exit 1; }
  echo "== $lib"; grep LNERF_PROF gpurun_out/pab.log | tail -1
done
