#!/bin/bash
# r05y: A/B of batch launches in the measured tile order (RT_BATCH_TILE_ORDER=1) -- golden check, then the
# driver's shape (--steps 20 --warmup 5) and 64-frame launches, C3 and C2, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05y
mkdir -p $O
RT_BATCH_TILE_ORDER=1 timeout -k 10 120 python - <<'PY' || exit 1
import json, zlib, sys
sys.path.insert(0, "uu-infogr-raytracer_amd")
import numpy as np, torch
from raytracer_hip import Context, abi, scenes
g = json.load(open("tests/golden/golden.json"))
for cid in ("C3", "C2"):
    sc = scenes.config(cid); W, H = sc.width, sc.height
    ctx = Context(1); ctx.set_scene(sc)
    big = torch.empty(4 * W * H, dtype=torch.int32, device="cuda")
    for rep in range(3):
        big.zero_()
        ctx.render_bands_batch(W, H, 8, 0, 1, 4, big.data_ptr(), W * H * 4, abi.RT_BANDS_FRAME, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        f = big.cpu().numpy().reshape(4, H, W)
        crcs = [f"{zlib.crc32(np.ascontiguousarray(x).tobytes()) & 0xffffffff:08x}" for x in f]
        assert all(c == g["cases"][cid]["crc32"] for c in crcs), (cid, rep, crcs)
    ctx.close()
print("batch tile order: golden C3/C2 frames, recording launch and sorted launches")
PY
for rep in 1 2 3; do
  for v in 0 1; do
    for cfg in C3 C2; do
      RT_BATCH_TILE_ORDER=$v timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 5 --also "" --no-cpu-baseline --no-tick \
          2> /dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('order=$v $cfg driver', round(d['value']/1e3,1), 'Gray/s', round(d['ms_per_step']*1e3,2), 'us')" >> $O/bench.txt || exit 1
    done
  done
done
for rep in 1 2; do
  for v in 0 1; do
    RT_BATCH_TILE_ORDER=$v timeout -k 10 200 python bench.py --config C3 --also "" --no-cpu-baseline --no-tick \
        2> /dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('order=$v C3 long', round(d['value']/1e3,1), 'Gray/s', round(d['ms_per_step']*1e3,2), 'us')" >> $O/bench.txt || exit 1
  done
done
cat $O/bench.txt
