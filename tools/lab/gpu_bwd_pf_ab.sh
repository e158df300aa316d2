# backward prefetch A/B: default build (dq / dK-dV score fragments read ahead behind fences) vs -DDKV_PF=0
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "attn or attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/bwdpf_tests.log 2>&1
tail -2 gpurun_out/bwdpf_tests.log
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pf_new$i -o run -- python3 tools/kbench.py attn > gpurun_out/prof_pf_new$i.log 2>&1
OBST_KERNELS=$PWD/bin/_kernels_pf0.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pf_old$i -o run -- python3 tools/kbench.py attn > gpurun_out/prof_pf_old$i.log 2>&1
done
grep -h pflops gpurun_out/prof_pf_*.log
