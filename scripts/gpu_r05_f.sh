#!/bin/bash
# Round 5: SMA bar segments combined in-kernel by the last speculative segment (config 5's
# shard): segment parity, then kernel time and HBM traffic, HEAD vs the round-4 library.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/c5
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_segments.py tests/test_gpu_fullsize.py -m gpu -k "sma or config5 or random" > gpurun_out/r05/c5/seg_tests.log 2>&1 || { tail -30 gpurun_out/r05/c5/seg_tests.log; exit 1; }
tail -1 gpurun_out/r05/c5/seg_tests.log
for lib in libbt.so dev/r4.so; do

  BT_LIB=$lib WORLD_SIZE=1 timeout -k 10 300 python3 bench.py --config 5 --symbols 1250 --scaling strong --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r05/c5/b_$lib.log 2>&1 || { tail -5 gpurun_out/r05/c5/b_$lib.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05/c5/b_$lib.log').read().strip().splitlines()[-1]); print('$lib config 5 shard kernel', round(d['roofline']['kernel_avg_ms'],2), 'ms/step', round(d['ms_per_step'],2), d['bar_segments'])"
  for pass in FETCH_SIZE WRITE_SIZE; do
    BT_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/r05/c5/${lib}_$pass -o p -- python3 bench.py --config 5 --symbols 1250 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r05/c5/pmc_${lib}_$pass.log 2>&1 || { echo "pmc $pass failed"; tail -5 gpurun_out/r05/c5/pmc_${lib}_$pass.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for lib in ("libbt.so", "dev/r4.so"):
    tot = {}
    for pass_ in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"gpurun_out/r05/c5/{lib}_{pass_}/**/*counter_collection.csv", recursive=True)
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f[0])):
            per[(r["Dispatch_Id"], r["Kernel_Name"].split("(")[0])] += float(r["Counter_Value"])
        # steady step = the last launch's kernels (dispatch ids of the final step)
        tot[pass_] = per
    for pass_, per in tot.items():
        byk = collections.defaultdict(list)
        for (d, k), v in per.items():
            byk[k].append((int(d), v))
        print(lib, pass_, {k.split("::")[-1][:24]: round(sorted(v)[-1][1] / 1024 ** 2, 1) for k, v in byk.items()}, "MiB (KiB units / 1024: last dispatch per kernel)")
PY
