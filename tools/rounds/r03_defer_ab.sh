#!/bin/bash
# A/B of the deferred speculative size check (RT_BENCH_NO_DEFER=1 = the host wait in the middle of the run), world-1
# rehearsal of the driver's shape, alternating, three times each, default path and rank 0 through the codec.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03dab
mkdir -p $O
line() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', round(d['ms_per_step']*1e3, 2), 'us/frame, verified', d.get('verified_frames'))"; }
for i in 1 2 3; do
  for mode in defer nodefer; do
    for path in direct codec; do
      F=""; [ $path = codec ] && F="--rank0-codec"
      E=""; [ $mode = nodefer ] && E=1
      RT_BENCH_NO_DEFER=$E timeout -k 10 200 python bench.py --dist-path $F --steps 20 --warmup 5 --verify --also-dist "" > $O/$path.$mode.$i.json 2> $O/$path.$mode.$i.err || { tail -20 $O/$path.$mode.$i.err; exit 1; }
      line $O/$path.$mode.$i.json "$path $mode $i"
    done
  done
done
