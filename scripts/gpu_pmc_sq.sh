# SQ stall/utilisation counters of the bench kernels (one PMC pass, kernel-trace off).
set -u
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d "$R/gpurun_out/pmc/sq" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/pmc/sq.log" 2>&1
echo "pmc rc=$?"
