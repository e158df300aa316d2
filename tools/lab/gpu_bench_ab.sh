# same-box headline A/B: the tree's kernels vs bin/_kernels_prev.so (the round's previous attention kernels)
set -e
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 | tail -1 | sed 's/^/new /' >> gpurun_out/bench_ab.log
  OBST_KERNELS=$PWD/bin/_kernels_prev.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 | tail -1 | sed 's/^/prev /' >> gpurun_out/bench_ab.log
done
cut -c1-140 gpurun_out/bench_ab.log
