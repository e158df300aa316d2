# activation GEMMs on gemm4w's fused epilogue (OBST_ACT_G4W=1) vs hipBLASLt + elementwise pass, same box
set -e
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 | tail -1 | sed 's/^/lt+ew /' >> gpurun_out/act_g4w_ab.log
  OBST_ACT_G4W=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 | tail -1 | sed 's/^/g4w_act /' >> gpurun_out/act_g4w_ab.log
done
cut -c1-130 gpurun_out/act_g4w_ab.log
