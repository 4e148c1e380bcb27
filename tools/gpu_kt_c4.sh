#!/bin/bash
R=$(pwd); O="$R/gpurun_out/r6_ramp_kt"; rm -rf "$O"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- $R/cop5615-gossip_protocol_amd/lib/gossip 100000000 full gossip > "$O/run.log" 2>&1
rc=$?; echo "rc=$rc"; tail -3 "$O/run.log"
python3 $R/tools/kt_summary.py "$O/kt/kt_kernel_trace.csv" > "$O/summary.txt"; head -20 "$O/summary.txt"
python3 - "$O/kt/kt_kernel_trace.csv" <<'PY' > "$O/seq.txt"
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
for r in rows[:400]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{(s-t0)/1e3:10.1f} {(e-s)/1e3:8.1f} {r["Kernel_Name"][:60]}')
PY
head -120 "$O/seq.txt"
