#!/bin/bash
# The torch.distributed path of bench.py at world 1 (RCCL communicator of the
# library, gpe_run_sharded_device, the C3 population-sharded leg).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r04}
DEAP_AMD_FORCE_DIST=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 \
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp32 --no-trig-leaves \
  > gpurun_out/${tag}_dist1.log 2>&1
rc=$?; echo "dist1 rc=$rc"; grep "^{" gpurun_out/${tag}_dist1.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['n_gpus'], json.dumps(r.get('c3_sharded')))"; exit $rc
