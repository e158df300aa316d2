"""round 6 debug: where does the flash map backward's dbias differ from the fp32 oracle (B=2 S=256 H=3 D=128)"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from homebrewnlp_mtf_amd.ops import raw
BF = torch.bfloat16
B, S, H, D = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), 128
causal = sys.argv[4] == "1"
torch.manual_seed(0)
q, k, v, do = [(torch.randn(B, S, H, D) * 0.7).to(BF) for _ in range(4)]
bias = torch.randn(H, S, S) * 0.5
res = {}
for dev in ("cpu", "cuda"):
    t = [x.to(dev).contiguous() for x in (q, k, v, do)]
    b = bias.to(dev)
    o = torch.zeros_like(t[0]); lse = torch.zeros(B * H * S, device=dev)
    raw.attn_map_fwd(t[0], t[1], t[2], o, lse, b, None, B, S, H, D, D ** -0.5, causal)
    o_in = res["cpu"][0].to(dev) if dev != "cpu" else o
    dq, dk, dv = (torch.zeros_like(t[0]) for _ in range(3))
    delta = torch.zeros(B * H * S, device=dev)
    db = torch.zeros(H, S, S, device=dev)
    pb = torch.full((B, H, S, S), float("nan"), device=dev) if dev != "cpu" else None
    raw.attn_map_bwd(t[0], t[1], t[2], o_in, t[3], lse, delta, dq, dk, dv, b, None, db, None, B, S, H, D, D ** -0.5,
                     causal, pb)
    res[dev] = (o, db.cpu(), pb.cpu() if pb is not None else None)
torch.cuda.synchronize()
g, c = res["cuda"][1], res["cpu"][1]
bad = (g - c).abs() > 5e-2 + 5e-2 * c.abs()
print("bad", int(bad.sum()), "of", bad.numel())
idx = bad.nonzero()
for hh in range(H):
    bh = bad[hh]
    if bh.any():
        qs, ks = bh.nonzero(as_tuple=True)
        print(f"h={hh} n={int(bh.sum())} q[{int(qs.min())},{int(qs.max())}] k[{int(ks.min())},{int(ks.max())}]")
        # rows / columns histogram
        print(" q rows hit:", sorted(set((qs // 16).tolist()))[:20], " k blocks:", sorted(set((ks // 16).tolist()))[:20])
print(idx[:10].tolist())
pbv = res["cuda"][2]
print("nan in part (causal lower):", int(torch.isnan(torch.tril(pbv.reshape(-1, S, S))).sum()))
print("sample g/c:", [(float(g[tuple(i)]), float(c[tuple(i)])) for i in idx[:5].tolist()])
ps = pbv.sum(0) if B > 1 else pbv[0]
ps = pbv.reshape(B, H, S, S).sum(0)
cm = torch.tril(torch.ones(S, S)) if causal else torch.ones(S, S)
for nm, cand in (("part-sum", ps * cm), ("part-sum^T", ps.transpose(-1, -2) * cm)):
    print(nm, "max err vs cpu", float((cand - c).abs().max()))
# per 16x16 / 4-row structure of one batch slab vs the oracle's batch-0 dS
qf, kf_, vf_, dof = (x.float() for x in (q, k, v, do))
s_ = torch.einsum("bqhd,bkhd->bhqk", qf, kf_) * D ** -0.5 + bias
if causal:
    s_ = s_.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool), 1), float("-inf"))
p_ = torch.softmax(s_, -1)
o_ = torch.einsum("bhqk,bkhd->bqhd", p_, vf_)
dp_ = torch.einsum("bqhd,bkhd->bhqk", dof, vf_)
dl_ = (dof * res["cpu"][0].float()).sum(-1).permute(0, 2, 1)
ds_ = p_ * (dp_ - dl_.unsqueeze(-1))
g0 = pbv.reshape(B, H, S, S)[0, 0]
r0 = ds_[0, 0]
print("slab0 err", float((g0 * cm - r0).abs().max()), "slab0^T err", float((g0.T * cm - r0).abs().max()))
for (qq, kk) in [(20, 3), (100, 40), (255, 0), (5, 5)]:
    print(qq, kk, float(g0[qq, kk]), float(r0[qq, kk]), float(r0[kk, qq]) if kk <= qq else None)
badm = ((g0 - r0).abs() > 1e-3 + 1e-2 * r0.abs()) & (cm > 0)
print("slab0 bad", int(badm.sum()), "of", int(cm.sum()))
for qb in range(S // 64):
    print("qblk", qb, [int(badm[qb*64:(qb+1)*64, kb*64:(kb+1)*64].sum()) for kb in range(S // 64)])
print("diag block rows 0..15, cols 0..15 bad:")
for qq in range(16):
    print("".join("X" if badm[qq, kk] else ("." if kk <= qq or not causal else " ") for kk in range(32)))
