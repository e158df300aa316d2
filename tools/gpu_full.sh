# round-end check: full GPU test suite, smoke(), headline bench, kernel profile of the headline step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_gpu.log 2>&1 || { echo "GPU tests failed"; tail -40 gpurun_out/full_gpu.log; exit 1; }
tail -2 gpurun_out/full_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_final.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log
bash tools/profile.sh final --steps 6 --warmup 3 > /dev/null 2>&1 || { echo "profile failed"; exit 1; }
head -24 gpurun_out/prof_final/steps.md
