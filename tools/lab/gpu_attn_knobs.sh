# attention knob sweep on one box: setprio bits (1 dK/dV, 2 dQ, 4 fwd) and the 8-wave forward
set -e
mkdir -p gpurun_out
for i in 1 2; do
for p in 1 0 3 5 7; do
  OBST_ATTN_PRIO=$p timeout -k 10 120 python -u tools/kbench.py attn | sed "s/^/prio$p /" >> gpurun_out/attn_knobs.log
done
OBST_ATTN_FWD_NW=8 timeout -k 10 120 python -u tools/kbench.py attn | sed "s/^/fwdnw8 /" >> gpurun_out/attn_knobs.log
done
cut -c1-200 gpurun_out/attn_knobs.log
