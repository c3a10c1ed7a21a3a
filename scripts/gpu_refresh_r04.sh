#!/bin/bash
# Round-4 evidence refresh: smoke, the driver's bench command (profiled: trace + PMC passes), the
# per-config shard profiles, and the default bench line with its CPU baseline; all under
# gpurun_out/ (summarised into profiles/r04/ by scripts/summarize_profile.py on the CPU side).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash scripts/gpu_profile.sh config2 --gpus 1 --steps 20 --warmup 5 || exit 1
bash scripts/gpu_profile_cfgs.sh || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-400
