#!/bin/bash
# Kernel trace of a short config-2 bench (per-kernel durations and the step timeline).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/tr
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr -o tr -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tr.log 2>&1 || exit $?
python3 - <<'PY'
import csv
rows = sorted(csv.DictReader(open("gpurun_out/tr/tr_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "_kernel" in r["Kernel_Name"] and "gen" not in r["Kernel_Name"]]
i = idx[-2]; t0 = int(rows[i]["Start_Timestamp"])
for r in rows[i:i + 10]:
    print(f'{r["Kernel_Name"][:44]:44s} {(int(r["Start_Timestamp"]) - t0) / 1e3:9.1f} {(int(r["End_Timestamp"]) - t0) / 1e3:9.1f} us')
PY
