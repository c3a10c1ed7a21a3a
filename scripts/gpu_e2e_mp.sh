#!/bin/bash
# gRPC-fed config-5 rehearsal with the counterparts in separate processes (scripts/e2e_grpc_mp.py)
# for each SPECS entry "workers:fetchers:jobs-per-request"; JSON lines under gpurun_out/e2e_mp/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/e2e_mp
for spec in ${SPECS:-1:4:16 2:4:16}; do
  IFS=: read w f b <<< "$spec"
  timeout -k 10 300 python3 -u scripts/e2e_grpc_mp.py --symbols ${SYMS:-256} --workers $w --fetchers $f --batch $b > gpurun_out/e2e_mp/w${w}_f${f}_b${b}.log 2>&1 || { tail -5 gpurun_out/e2e_mp/w${w}_f${f}_b${b}.log; exit 1; }
  tail -1 gpurun_out/e2e_mp/w${w}_f${f}_b${b}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('workers', d['workers'], 'fetchers', d['fetchers'], 'batch', d['batch'], 'wall', round(d['wall_s'],2), 'GB/s', round(d['GBps'],3), 'all_done', d['all_done'])"
done
