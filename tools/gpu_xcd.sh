# XCD-contiguous block order (MM_XCD_REMAP=1) for the wide kernel: time and read traffic
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/xcd
mkdir -p $R
for x in 0 1; do
  for spec in "20:5" "96:16"; do
    IFS=: read steps warm <<< "$spec"
    OUT=$R/x${x}_s$steps; mkdir -p $OUT
    MM_XCD_REMAP=$x timeout -k 10 200 python3 -u bench.py --steps $steps --warmup $warm --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
    tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('x=$x steps=$steps', d['value'], d['roofline']['kernel_avg_us'])"
    MM_XCD_REMAP=$x timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --steps $steps --warmup $warm --no-cpu-baseline > $OUT/fetch.log 2>&1 || { echo "fetch rc=$?"; tail $OUT/fetch.log; exit 1; }
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
