# The driver's timed region vs its kernel: rocprofv3 kernel-trace timestamps of
# tools/timed_gap.py (bench sequence, back to back, after idle) -- is the first timed K = 20
# pass itself longer, or does something sit between the launch and the kernel.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/gaptrace}
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run -- python3 tools/timed_gap.py > $D/gap.log 2>&1 || { tail -20 $D/gap.log; exit 1; }
cat $D/gap.log
python3 - $D <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/trace/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"][:60]
    gap = (s - prev) / 1e3 if prev else 0
    print(f"{name:60s} dur_us={(e - s) / 1e3:9.1f} gap_from_prev_end_us={gap:9.1f}")
    prev = e
PY
