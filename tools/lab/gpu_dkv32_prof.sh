# per-kernel times of the attention backward: default dK/dV kernel vs the pipelined 32x32 one (OBST_ATTN_BWD=2)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bwd1 -o run -- python3 tools/kbench.py attn > gpurun_out/prof_bwd1.log 2>&1
OBST_ATTN_BWD=2 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bwd2 -o run -- python3 tools/kbench.py attn > gpurun_out/prof_bwd2.log 2>&1
for v in 1 2; do f=$(find gpurun_out/prof_bwd$v -name '*kernel_stats.csv' | head -1); echo "== bwd$v"; grep -i attn "$f" | cut -d, -f1-5; done
