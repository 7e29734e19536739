#!/bin/bash
# One-process rehearsal of the N > 1 path (RCCL world of 1, rank 0 through the codec): frame period
# of the driver's short command and of a long run, with and without speculative gather sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for steps in "20 5" "1024 256"; do
  set -- $steps
  for spec in "" "--no-speculate"; do
    for rep in 1 2; do
      timeout -k 10 120 python bench.py --dist-path --rank0-codec --steps $1 --warmup $2 --no-cpu-baseline $spec 2>/dev/null \
        | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('steps', d['steps'], '$spec' or 'speculative', round(d['ms_per_step']*1e3,2), 'us/frame', 'host', round(d['host_ms_per_step']*1e3,2), 'redone', d['config'].get('gather_redone_batches'))" || exit 1
    done
  done
done
