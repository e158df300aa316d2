"""round 6: per-block phase clocks of the token-mixer GEMMs (gemm4w stamps: loop / epilogue clocks per tile, block
busy time vs launch span) at kbench's mixer shape, against a dense GEMM of similar size.
  python tools/lab/mixer_stamps.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from homebrewnlp_mtf_amd.ops import _lib as L, raw  # noqa: E402

BF = torch.bfloat16


def stamped(fn, label, kt_per_tile=None):
    lib = L.lib()
    lib.obst_gemm4w_stamps.argtypes = [ctypes.c_void_p]
    lib.obst_gemm4w_stamps.restype = None
    st = torch.zeros(256 * 8, dtype=torch.int64, device="cuda")
    fn()
    torch.cuda.synchronize()
    lib.obst_gemm4w_stamps(st.data_ptr())
    fn()
    torch.cuda.synchronize()
    lib.obst_gemm4w_stamps(None)
    h = st.view(256, 8).cpu().tolist()
    rows = [t for t in h if t[6]]
    nb = len(rows)
    tiles = sum(t[7] for t in rows)
    loop = sum(t[2] for t in rows)
    s1 = sum(t[0] for t in rows)
    s2 = sum(t[1] for t in rows)
    epi = sum(t[3] for t in rows)
    span = (max(t[6] for t in rows) - min(t[5] for t in rows)) / 100.0
    busy = [(t[6] - t[5]) / 100.0 for t in rows]
    print(f"{label}: {nb} blocks, {tiles / nb:.1f} tiles/block, per tile: loop {loop / tiles:.0f} clk"
          + (f" ({loop / tiles / kt_per_tile:.0f} per K-tile)" if kt_per_tile else "")
          + f" [barrier waits: LDS-read {s1 / tiles:.0f}, DMA-landed {s2 / tiles:.0f}]"
          + f", epilogue {epi / tiles:.0f} clk; block busy mean {sum(busy) / nb:.1f} min {min(busy):.1f} max "
          f"{max(busy):.1f} us; launch span {span:.1f} us")
    # timing without stamps
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"   {label}: {e0.elapsed_time(e1) / 10 * 1000:.1f} us per call (no stamps)")


def main():
    B, S, H, Fd = 32, 2048, 8, 256
    x = (torch.randn(B * S * H * Fd, device="cuda") * 0.5).to(BF)
    w = torch.tril((torch.randn(H, S, S, device="cuda") * 0.05)).to(BF).reshape(-1)
    y = torch.empty_like(x)
    hf = H * Fd
    for name, a_t, tri in (("mixer y", 0, 1), ("mixer dx", 1, 2)):
        stamped(lambda: raw.gemm(raw.Operand(w, a_t, S, 0, S * S), raw.Operand(x, 1, hf, S * hf, Fd),
                                 raw.Operand(y, 0, hf, S * hf, Fd), S, Fd, S, batch=(B, H), tri=tri),
                name, kt_per_tile=18.0)
    # the same product untriangled (dense K = 2048 per tile) and a plain dense GEMM of the step
    stamped(lambda: raw.gemm(raw.Operand(w, 0, S, 0, S * S), raw.Operand(x, 1, hf, S * hf, Fd),
                             raw.Operand(y, 0, hf, S * hf, Fd), S, Fd, S, batch=(B, H), tri=0),
            "mixer y dense", kt_per_tile=32.0)
    M, N = 16384, 8192
    for K in (512, 1024, 4096):
        a = (torch.randn(M * K, device="cuda")).to(BF)
        b = (torch.randn(N * K, device="cuda")).to(BF)
        c = torch.empty(M * N, device="cuda", dtype=BF)
        stamped(lambda: raw.gemm(raw.Operand(a, 0, K), raw.Operand(b, 0, K), raw.Operand(c, 0, N), M, N, K),
                f"dense {M}x{N}x{K} (B K-contiguous)", kt_per_tile=K / 64)
    K = 2048
    a = (torch.randn(M * K, device="cuda")).to(BF)
    b = (torch.randn(N * K, device="cuda")).to(BF)
    c = torch.empty(M * N, device="cuda", dtype=BF)
    stamped(lambda: raw.gemm(raw.Operand(a, 0, K), raw.Operand(b, 1, N), raw.Operand(c, 0, N), M, N, K),
            "dense 16384x8192x2048 (B row-contiguous)", kt_per_tile=32.0)
    stamped(lambda: raw.gemm(raw.Operand(a, 0, K), raw.Operand(b, 0, K), raw.Operand(c, 0, N), M, N, K),
            "dense 16384x8192x2048 (B K-contiguous)", kt_per_tile=32.0)


if __name__ == "__main__":
    main()
