#!/bin/bash
# r05p: round-5 evidence for the C3 headline -- PMC passes + kernel trace reconcile per config (C3 first; the
# traffic table profiles/pmc_traffic.json gains C3's entry), then copies the summaries to gpurun_out/r05p.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05p
mkdir -p $O
bash tools/profile_round.sh ${CFGS:-C3 C2 C4 C5} || exit 1
for c in ${CFGS:-C3 C2 C4 C5}; do
  cp gpurun_out/pmc_${c}_summary.txt gpurun_out/trace_${c}_reconcile.txt gpurun_out/trace_bench_$c.json \
     gpurun_out/trace_${c}_kernel_stats.csv $O/ 2>/dev/null
done
cp gpurun_out/pmc_traffic.json $O/
for f in $O/trace_*_reconcile.txt; do tail -n 2 $f; done
