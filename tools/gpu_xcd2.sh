# XCD chunk order (MM_XCD_CHUNK) for the wide kernel: kernel time and read traffic, and the
# K = 16 / 20 pass times at 32768^2 and 16384^2 (planner cost table)
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/xcd2
mkdir -p $R
timeout -k 10 300 python3 -u tools/kernel_table.py --sizes 32768x32768,16384x16384 --old 8 --wide 12,16,20 > $R/kernel_table.log 2>&1 || { tail $R/kernel_table.log; exit 1; }
cat $R/kernel_table.log
for c in 0 16 32 64; do
  for spec in "20:5" "96:16"; do
    IFS=: read steps warm <<< "$spec"
    OUT=$R/c${c}_s$steps; mkdir -p $OUT
    MM_XCD_CHUNK=$c timeout -k 10 200 python3 -u bench.py --steps $steps --warmup $warm --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
    tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunk=$c steps=$steps', d['value'], d['roofline']['kernel_avg_us'])"
    MM_XCD_CHUNK=$c timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --steps $steps --warmup $warm --no-cpu-baseline > $OUT/fetch.log 2>&1 || { echo "fetch rc=$?"; tail $OUT/fetch.log; exit 1; }
    python3 - $OUT <<'PY'
import csv, glob, sys, statistics
rows = []
for f in glob.glob(sys.argv[1] + "/fetch/**/*counter_collection.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if "mm_wide_kernel" in r.get("Kernel_Name", "")]
by = {}
for r in rows:
    by.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
for k, v in by.items():
    print("  FETCH bytes/launch (x2)", round(2 * statistics.mean(v) * 1024 / 1e9, 3), "GB", len(v), k[:70])
PY
  done
done
