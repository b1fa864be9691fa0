"""Per-parameter gradient error of the bf16 path vs the fp32 path and the oracle."""
import sys
import torch
sys.path.insert(0, ".")
import two_towers_amd as tta
from oracle import cpu_ref

E, h, B, T = 64, 32, 96, 10
torch.manual_seed(1)
m = tta.EnhancedTwoTowerModel(E, h)
p = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
m = m.cuda().eval()
g = torch.Generator().manual_seed(6)
q = torch.randn(B, T, E, generator=g)
d = torch.randn(B, T, E, generator=g)
grads = {}
for dt in (torch.float32, torch.bfloat16):
    m.zero_grad()
    m.set_compute_dtype(dt)
    qv, dv = m(q.cuda(), d.cuda())
    loss = tta.InfoNCELoss(compute_dtype=dt)(qv, dv)
    loss.backward()
    grads[dt] = {k: v.grad.detach().cpu().clone() for k, v in m.named_parameters()}
    print(dt, "loss", float(loss))
rl = cpu_ref.infonce(*cpu_ref.forward(q, d, p))
rl.backward()
print("oracle loss", float(rl))
for k in p:
    a, b, r = grads[torch.bfloat16][k].double(), grads[torch.float32][k].double(), p[k].grad.double()
    mr = float((a - r).abs().max() / r.abs().max())
    fr = float((a - r).norm() / r.norm())
    cos = float((a * r).sum() / (a.norm() * r.norm()))
    f32 = float((b - r).norm() / r.norm())
    print(f"{k:40s} bf16 maxrel {mr:.4f} frob {fr:.4f} cos {cos:.5f} | fp32 frob {f32:.2e}")
