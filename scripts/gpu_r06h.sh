# round-6 session h: why k2 on fp16-planes A slabs runs slower -- exceptional-row counts and kernel
# times of the product and the planes build
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/loma-nerf_amd/lib
for lib in libloma_nerf libloma_nerf_ap; do
  LNERF_LIB=$L/$lib.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-render --no-cfg2 --no-cpu-baseline \
    > gpurun_out/bh_$lib.log 2>&1 || { tail -5 gpurun_out/bh_$lib.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bh_$lib.log') if l.startswith('{')][-1])
print('$lib', d['ms_per_step'], d['kernels_ms'], d.get('exceptional_rows'))"
done
