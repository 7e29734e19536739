#!/bin/bash
# GPU box: codec parity tests, isolated codec timings and their kernel-trace summary, then the
# one-process rehearsal of the N>1 path (DIST_RUNS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_parity.py -k "codec or band or traced" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
PROFILE=1 bash tools/codec_bench.sh > /dev/null 2>&1
grep world gpurun_out/codec_bench.txt
find gpurun_out/prof_codec -name "*kernel_stats.csv" -exec cat {} \; | python3 -c "
import csv,sys
for r in csv.DictReader(sys.stdin):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us avg')" | grep -v Fill
[ -n "${DIST_RUNS:-}" ] && bash tools/dist_rehearsal.sh
exit 0
