#!/bin/bash
# r05z: A/B of bundle-kernel lone frames in the measured tile order (RT_BUNDLE_TILE_ORDER=1): golden check,
# then one-frame launches of C4 / C5 (counters off), H = the previous commit's library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05z
mkdir -p $O
RT_BUNDLE_TILE_ORDER=1 timeout -k 10 120 python - <<'PY' || exit 1
import json, zlib, sys
sys.path.insert(0, "uu-infogr-raytracer_amd")
import numpy as np, torch
from raytracer_hip import Context, scenes
g = json.load(open("tests/golden/golden.json"))
for cid in ("C4", "C5"):
    sc = scenes.config(cid); W, H = sc.width, sc.height
    ctx = Context(1); ctx.set_scene(sc)
    out = torch.empty(W * H, dtype=torch.int32, device="cuda")
    for rep in range(3):
        out.zero_()
        ctx.render_device(W, H, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        c = f"{zlib.crc32(np.ascontiguousarray(out.cpu().numpy()).tobytes()) & 0xffffffff:08x}"
        assert c == g["cases"][cid]["crc32"], (cid, rep, c)
    ctx.close()
print("bundle tile order: golden C4/C5 frames, recording launch and sorted launches")
PY
for c in C4 C5; do
  for rep in 1 2; do
    for v in "H|0" "T|0" "T|1"; do
      lib=lib/libraytracer_hip.so; [ ${v%%|*} = H ] && lib=lib/ab/libraytracer_hip_H.so
      RT_BUNDLE_TILE_ORDER=${v#*|} timeout -k 10 180 python tools/frame_wall.py --config $c --batch 1 --frames $([ $c = C5 ] && echo 256 || echo 1024) --no-count \
          --lib uu-infogr-raytracer_amd/$lib 2>&1 | grep -v amdgpu.ids | sed "s/^/$v: /" >> $O/wall.txt || exit 1
    done
  done
done
sed 's/strip=- bands=- //; s/host enqueue.*//' $O/wall.txt
