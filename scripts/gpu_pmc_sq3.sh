# SQ counters of the bench kernels, three passes (each pass within the per-block slot limits),
# summed per kernel name: utilisation, instruction mix, LDS activity.
set -u
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmc"; rm -rf "$R/gpurun_out/pmc/p"*
cd /tmp && export TMPDIR=/tmp
LIBARG=""
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_ANY"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/pmc/p$i.log"; exit 1; }
done
python3 - "$R" <<'PY'
import csv, collections, sys, glob
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob(sys.argv[1] + "/gpurun_out/pmc/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("lnerf::(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        if "k16_fwd" in k or "kact" in k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]] += 1
for k, d in agg.items():
    print(k)
    for c in sorted(d):
        print("   %-28s %.4g (per dispatch-row avg over %d rows)" % (c, d[c] / max(1, cnt[k][c]) , cnt[k][c]))
PY
