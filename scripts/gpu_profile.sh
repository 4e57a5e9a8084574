# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE / WRITE_SIZE) of the bench.
set -u
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/prof"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 10 --warmup 3 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/trace" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof/trace.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof/fetch" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof/fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/prof/write" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof/write.log" 2>&1
echo "profile rc=$?"
find "$R/gpurun_out/prof" -name "*.csv" | head -20
