# One GPU session = a list of named steps, each under its own time limit, stopping at the first
# failure (a fault, abort, time limit or failing test ends the call):
#   gpurun -- bash scripts/gpu_steps.sh tests bench trace sq
# steps: tests | bench | dist | render | precision | trace | pmc | sq | compat
# Logs go to gpurun_out/<step>.log; rocprof output under gpurun_out/prof and gpurun_out/sq.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
        --timeout-method thread > gpurun_out/tests.log 2>&1
      rc=$?; tail -3 gpurun_out/tests.log ;;
    bench)
      timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
      rc=$?; tail -1 gpurun_out/bench.log | cut -c1-900 ;;
    dist)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v -p no:cacheprovider \
        --timeout 120 --timeout-method thread > gpurun_out/dist.log 2>&1 &&
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29517 bench.py --no-cpu-baseline \
        > gpurun_out/dist_weak.log 2>&1 &&
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29518 bench.py --strong --no-cpu-baseline \
        > gpurun_out/dist_strong.log 2>&1
      rc=$?; tail -3 gpurun_out/dist.log; tail -1 gpurun_out/dist_weak.log | cut -c1-400
      tail -1 gpurun_out/dist_strong.log | cut -c1-400 ;;
    render)
      timeout -k 10 300 python bench.py --render --steps 5 --warmup 2 > gpurun_out/render.log 2>&1
      rc=$?; tail -1 gpurun_out/render.log | cut -c1-500 ;;
    precision)
      timeout -k 10 300 python scripts/precision_report.py > gpurun_out/precision.log 2>&1
      rc=$?; tail -8 gpurun_out/precision.log ;;
    compat)
      timeout -k 10 300 python scripts/bench_compat.py > gpurun_out/compat.log 2>&1
      rc=$?; tail -4 gpurun_out/compat.log ;;
    trace)
      mkdir -p gpurun_out/prof
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$R/gpurun_out/prof/trace" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 \
        --no-cpu-baseline --no-render > "$R/gpurun_out/prof/trace.log" 2>&1)
      rc=$? ;;
    pmc)
      mkdir -p gpurun_out/prof
      (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d "$R/gpurun_out/prof/fetch" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 \
        --no-cpu-baseline --no-render > "$R/gpurun_out/prof/fetch.log" 2>&1) &&
      (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv \
        -d "$R/gpurun_out/prof/write" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 \
        --no-cpu-baseline --no-render > "$R/gpurun_out/prof/write.log" 2>&1)
      rc=$? ;;
    sq)
      bash scripts/gpu_sq.sh
      rc=$? ;;
    *)
      echo "unknown step $step"; rc=2 ;;
  esac
  echo "step $step rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
