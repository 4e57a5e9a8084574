# One GPU session = a list of named steps, each under its own time limit, stopping at the first
# failure (a fault, abort, time limit or failing test ends the call):
#   gpurun -- bash scripts/gpu_steps.sh tests bench trace sq
# steps: tests | bench | dist | render | precision | trace | pmc | sq | rtrace | rpmc | rsq | compat
# (r*: the same profiles of the config-5 render, bench.py --render, under gpurun_out/rprof, rsq)
# Logs go to gpurun_out/<step>.log; rocprof output under gpurun_out/prof and gpurun_out/sq.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
lib_sha() { python3 -c "import hashlib,sys; print(hashlib.sha256(open(sys.argv[1],'rb').read()).hexdigest()[:16])" \
  "${LNERF_LIB:-$R/loma-nerf_amd/lib/libloma_nerf.so}"; }
for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
        --timeout-method thread > gpurun_out/tests.log 2>&1
      rc=$?; tail -3 gpurun_out/tests.log ;;
    bench)
      timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
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
    trace|rtrace)
      # rocprofv3 kernel trace + stats of the training bench (trace) or the config-5 render (rtrace)
      if [ "$step" = trace ]; then D="$R/gpurun_out/prof"; A="--steps 10 --warmup 3 --no-cpu-baseline --no-render --no-cfg2"
      else D="$R/gpurun_out/rprof"; A="--render --steps 5 --warmup 2"; fi
      mkdir -p "$D"; echo "python3 bench.py $A" > "$D/command.txt"; lib_sha > "$D/lib_sha16.txt"
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$D/trace" -o run -- python3 "$R/bench.py" $A > "$D/trace.log" 2>&1)
      rc=$? ;;
    pmc|rpmc)
      if [ "$step" = pmc ]; then D="$R/gpurun_out/prof"; A="--steps 10 --warmup 3 --no-cpu-baseline --no-render --no-cfg2"
      else D="$R/gpurun_out/rprof"; A="--render --steps 3 --warmup 1"; fi
      mkdir -p "$D"; echo "python3 bench.py $A" > "$D/command.txt"; lib_sha > "$D/lib_sha16.txt"
      (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d "$D/fetch" -o run -- python3 "$R/bench.py" $A > "$D/fetch.log" 2>&1) &&
      (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv \
        -d "$D/write" -o run -- python3 "$R/bench.py" $A > "$D/write.log" 2>&1)
      rc=$? ;;
    sq)
      bash scripts/gpu_sq.sh "$R/gpurun_out/sq" --steps 3 --warmup 1 --no-cpu-baseline --no-render --no-cfg2
      rc=$? ;;
    rsq)
      bash scripts/gpu_sq.sh "$R/gpurun_out/rsq" --render --steps 2 --warmup 1
      rc=$? ;;
    *)
      echo "unknown step $step"; rc=2 ;;
  esac
  echo "step $step rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
