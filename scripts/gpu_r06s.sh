# round-6 session s: the driver's round-end steps on the final tree -- build check (no rebuild), smoke(),
# the default bench line
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_s.log 2>&1
rc=$?; tail -1 gpurun_out/bench_s.log | cut -c1-400; exit $rc
