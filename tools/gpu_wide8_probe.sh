# C = 8 vs C = 4 level-split kernel at K = 8 (tools/wide8_probe): time, SQ split, LDS and TA counters
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/w8probe
mkdir -p $R
timeout -k 10 120 tools/wide8_probe 0 5 > $R/time.log 2>&1 || { cat $R/time.log; exit 1; }
cat $R/time.log
for c in 4 8; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $R/sq$c -o run -- tools/wide8_probe $c 3 > $R/sq$c.log 2>&1 || { echo "sq$c rc=$?"; tail -5 $R/sq$c.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL TA_BUSY_avr --output-format csv -d $R/lds$c -o run -- tools/wide8_probe $c 3 > $R/lds$c.log 2>&1 || { echo "lds$c rc=$?"; tail -5 $R/lds$c.log; }
done
python3 - <<'PY'
import csv, glob, collections
for c in (4, 8):
    for kind in ("sq", "lds"):
        rows = []
        for f in glob.glob(f"gpurun_out/w8probe/{kind}{c}/**/*counter_collection.csv", recursive=True):
            rows += list(csv.DictReader(open(f)))
        agg = collections.defaultdict(list)
        for r in rows:
            if "mm_wide_kernel" in r.get("Kernel_Name", ""):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(c, kind, {k: round(sum(v) / len(v)) for k, v in agg.items()})
PY
