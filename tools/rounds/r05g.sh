#!/bin/bash
# r05g: round check after the ABI 9 Tick and the C3 headline (tools/round_check.sh), then the N = 2 rehearsal
# on this one GPU (two ranks over gloo; rank 0's single-process plugin-Tick leg on shared-device workers).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash tools/round_check.sh gpurun_out/r05g || exit 1
timeout -k 10 300 python bench.py --gpus 2 --rehearse-gloo --steps 20 --warmup 5 --no-cpu-baseline --master-port 29611 \
    > gpurun_out/r05g/rehearse2.json 2> gpurun_out/r05g/rehearse2.err || { tail gpurun_out/r05g/rehearse2.err; exit 1; }
python3 -c "
import json; d = json.loads(open('gpurun_out/r05g/rehearse2.json').read().strip().splitlines()[-1])
print('rehearse2', d['config']['workload'][:3], round(d['value']/1e3,1), 'Gray/s verified', d.get('verified_frames'), 'plugin_tick', json.dumps(d.get('plugin_tick'))[:600])"
