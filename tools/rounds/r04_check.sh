set -o pipefail
mkdir -p gpurun_out/r04a
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04a/gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/r04a/gpu.log; exit 1; }
tail -3 gpurun_out/r04a/gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04a/smoke.log 2>&1 || { cat gpurun_out/r04a/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r04a/bench.json 2> gpurun_out/r04a/bench.err || { tail gpurun_out/r04a/bench.err; exit 1; }
echo BENCH OK
