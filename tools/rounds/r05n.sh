#!/bin/bash
# r05n: rank 0's measured share in the N > 1 pipeline, rehearsed on one GPU (gloo ranks sharing it): the GPU
# paths' rehearsal tests, then the driver's shape at N = 3 / 8 for C3 and C5 (rank0-share auto, verified).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_paths.py -x -q --timeout 120 --timeout-method thread -k "rehearsal" > $O/rehearsal_tests.log 2>&1 \
    || { echo "REHEARSAL TESTS FAILED"; tail -40 $O/rehearsal_tests.log; exit 1; }
echo "rehearsal tests: $(tail -1 $O/rehearsal_tests.log)"
for n in 3 8; do
  timeout -k 10 300 python bench.py --gpus $n --rehearse-gloo --steps 20 --warmup 5 --no-cpu-baseline --no-tick \
      --master-port $((29700 + n)) > $O/rehearse$n.json 2> $O/rehearse$n.err || { tail -20 $O/rehearse$n.err; exit 1; }
  grep "share" $O/rehearse$n.err | head -4
  python3 -c "
import json; d = json.loads(open('$O/rehearse$n.json').read().strip().splitlines()[-1])
print('N=$n', d['config']['workload'][:3], 'verified', d.get('verified_frames'), d['config']['parallelism'][:160])
for k, v in d.get('also', {}).items(): print('   also', k, 'verified', v.get('verified_frames'), v['config'].get('rank0_tail_rows'))"
done
