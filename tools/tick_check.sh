cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?
echo "pytest rc=$rc: $(tail -1 gpurun_out/pt.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 64 > gpurun_out/b.log 2>&1 || exit $?
grep -h "^{" gpurun_out/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["tick_fps_incl_d2h"], d["tick_async_fps_incl_d2h"])'
timeout -k 10 200 python tools/tick_probe.py > gpurun_out/tick_probe.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/tick_probe.txt; exit $rc
