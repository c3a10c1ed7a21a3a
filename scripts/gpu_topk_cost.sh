# Kernel time and step time of the config-2 bench with and without the top-k chain (interference
# of the chain, which overlaps the next step's kernel on its own stream).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for t in 100 0 100 0; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --topk $t > gpurun_out/tk.log 2>&1 || { tail -3 gpurun_out/tk.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/tk.log').read().strip().splitlines()[-1]); print('topk', $t, round(d['roofline']['kernel_avg_ms'],4), round(d['ms_per_step'],4))"
done
