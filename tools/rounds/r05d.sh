#!/bin/bash
# r05d: tools/probes/exit_abort_probe.py, one sequence per process (exit status of each)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
for s in ${SEQS:-A B C D E F}; do
  timeout -k 10 120 python tools/probes/exit_abort_probe.py $s > /tmp/p_$s.log 2>&1
  echo "$s rc=$? $(tail -2 /tmp/p_$s.log | tr '\n' ' ')"
done
