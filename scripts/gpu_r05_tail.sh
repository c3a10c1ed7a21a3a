cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/tail
for s in 4608 5000 5376 4992 3840; do
  timeout -k 10 200 python3 bench.py --symbols $s --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05/tail/b_$s.log 2>&1 || { tail -5 gpurun_out/r05/tail/b_$s.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05/tail/b_$s.log').read().strip().splitlines()[-1]); k=d['roofline']['kernel_avg_ms']; print($s, 'kernel', round(k,4), 'us/symbol', round(1000*k/$s,4))"
done
