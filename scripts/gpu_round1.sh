# GPU tests, the default bench, and an RCCL rehearsal of the data-parallel bench path (torchrun, 1 rank).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t1.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-rays 16 > gpurun_out/b1.log 2>&1
  brc=$?
  echo "bench rc=$brc" >> gpurun_out/b1.log
  if [ $brc -eq 0 ]; then
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b_dist.log 2>&1
    echo "dist bench rc=$?" >> gpurun_out/b_dist.log
  fi
fi
tail -30 gpurun_out/t1.log
tail -5 gpurun_out/b1.log
tail -3 gpurun_out/b_dist.log 2>/dev/null
exit 0
