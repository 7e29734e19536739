set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python tools/region_probe.py --order 0s,0p,0s > gpurun_out/rp_base.txt 2>&1 &&
timeout -k 10 120 python tools/region_probe.py --order 0s,0p,0s --spin > gpurun_out/rp_spin.txt 2>&1 &&
ROC_ACTIVE_WAIT_TIMEOUT=2000 timeout -k 10 120 python tools/region_probe.py --order 0s,0p,0s > gpurun_out/rp_awt.txt 2>&1
grep -v amdgpu.ids gpurun_out/rp_*.txt
