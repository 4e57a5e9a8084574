# quick iteration: GPU tests, precision report, bench (each step under its own time limit)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t1.log
tail -25 gpurun_out/t1.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python scripts/precision_report.py > gpurun_out/prec.log 2>&1 && tail -6 gpurun_out/prec.log &&
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b1.log 2>&1
  echo "bench rc=$?"; tail -2 gpurun_out/b1.log
  if [ -f loma-nerf_amd/lib/libloma_nerf_prof.so ]; then
    LNERF_LIB=loma-nerf_amd/lib/libloma_nerf_prof.so timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bprof.log 2>&1
    grep LNERF_PROF gpurun_out/bprof.log | tail -1
  fi
fi
exit 0
