set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t1.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-rays 8 > gpurun_out/b1.log 2>&1
  echo "bench rc=$?" >> gpurun_out/b1.log
fi
tail -30 gpurun_out/t1.log
tail -5 gpurun_out/b1.log
