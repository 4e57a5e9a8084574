# L2 hit/miss counters of the bench kernels (one PMC pass).
set -u
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d "$R/gpurun_out/pmc/l2" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/pmc/l2.log" 2>&1
echo "pmc rc=$?"
python3 - "$R" <<'PY'
import csv, collections, sys
rows = list(csv.DictReader(open(sys.argv[1] + "/gpurun_out/pmc/l2/run_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in rows:
    k = r["Kernel_Name"].split("(")[0][-40:]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "k16" in k or "dw_all" in k:
        print(k, {c: "%.3g" % v for c, v in d.items()})
PY
