# SQ / GRBM counters of the bench kernels: three PMC passes of the same bench command, each within
# the per-block slot limits of MI355X_MICROARCH.md (<= 8 SQ, <= 2 GRBM), each its own run under
# its own time limit; scripts/summarize_sq.py turns gpurun_out/sq/ into profiles/<tag>_sq.json.
#   bash scripts/gpu_sq.sh OUT_DIR bench.py-args...
set -u
R="$GRAFT_REPO_ROOT"
OUT="$1"; shift
mkdir -p "$OUT"; rm -rf "$OUT"/p*
echo "python3 bench.py $*" > "$OUT/command.txt"
python3 -c "import hashlib,sys; print(hashlib.sha256(open(sys.argv[1],'rb').read()).hexdigest()[:16])" \
  "${LNERF_LIB:-$R/loma-nerf_amd/lib/libloma_nerf.so}" > "$OUT/lib_sha16.txt"
# the render runs plain bf16 MFMAs: count those instead of the fp16 ones
case " $* " in *" --render "*) MOPS=SQ_INSTS_VALU_MFMA_MOPS_BF16 ;; *) MOPS=SQ_INSTS_VALU_MFMA_MOPS_F16 ;; esac
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU $MOPS SQ_WAVES"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$R/bench.py" "$@" > "$OUT/p$i.log" 2>&1 \
    || { echo "sq pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "sq pass $i ok"
done
