#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
timeout -k 10 200 python -u bench.py --workloads c5 --no-cpu-baseline > $O/c5chk_plain_$i.json 2> $O/c5chk_plain_$i.err; echo "plain $i rc=$?"
done
timeout -k 10 300 python -u bench.py --e2e --workloads c5 --no-cpu-baseline > $O/c5chk_e2e.json 2> $O/c5chk_e2e.err; echo "e2e rc=$?"
VXG_PLAN_BATCH=0 timeout -k 10 300 python -u bench.py --e2e --workloads c5 --no-cpu-baseline > $O/c5chk_e2e_b0.json 2> $O/c5chk_e2e_b0.err; echo "e2e batch0 rc=$?"
exit 0
