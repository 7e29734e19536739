#!/bin/bash
# Deferred speculative size check (one-batch N>1 runs): world-1 rehearsal of the driver's shape, every frame verified,
# default path and rank 0 through the codec, plus the GPU tests of the pipeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03df
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --dist-path --steps 20 --warmup 5 --verify --also-dist "" > $O/direct_$i.json 2> $O/direct_$i.err || { tail -20 $O/direct_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/direct_$i.json') if l.startswith('{')][-1]); print('direct', d['ms_per_step']*1e3, 'us/frame', round(d['value']), 'verified', d.get('verified_frames'), d.get('gather'))"
done
timeout -k 10 300 python bench.py --dist-path --rank0-codec --steps 20 --warmup 5 --verify --also-dist "" > $O/codec.json 2> $O/codec.err || { tail -20 $O/codec.err; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open('$O/codec.json') if l.startswith('{')][-1]); print('codec', d['ms_per_step']*1e3, 'us/frame', round(d['value']), 'verified', d.get('verified_frames'), d.get('gather'))"
grep -h "repeated" $O/*.err || true
