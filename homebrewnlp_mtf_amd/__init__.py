"""homebrewnlp_mtf_amd -- an MI355X-native (gfx950 / CDNA4) re-design of HomebrewNLP-MTF ("OBST").

Layers:
  config.py        L1  JSON ModelParameter
  models/          L3  block grammar, layers, reversible bodies, model assembly
  ops/             L2  autograd ops backed by hand-written HIP kernels (csrc/kernels) with a torch CPU oracle
  optim/           L4  optimizer chain (SM3/Adam/NovoGrad/Adafactor/...), LR schedules, fused flat-buffer step
  parallel/        --  Mesh(dp, tp), RCCL collectives, bucketed DP gradient all-reduce
  data/            L5  native TFRecord reader, windowing, rank sharding, resume, pinned prefetch
  run/             L6/L7 train loop, sampling, query/debug/web_api run modes
  utils/           checkpointing, metrics, logging, profiling
"""
__version__ = "0.1.0"
