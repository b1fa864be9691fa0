"""bf16 path vs fp32 oracle evaluated on bf16-ROUNDED inputs and weights: isolates
the kernels' internal rounding from the sensitivity to input/weight quantisation."""
import sys
import torch
sys.path.insert(0, ".")
import two_towers_amd as tta
from oracle import cpu_ref

E, h, B, T = 64, 32, 96, 10
torch.manual_seed(1)
m = tta.EnhancedTwoTowerModel(E, h)
with torch.no_grad():
    for p in m.parameters():
        p.copy_(p.to(torch.bfloat16).float())
p = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
m = m.cuda().eval().set_compute_dtype(torch.bfloat16)
g = torch.Generator().manual_seed(6)
q = torch.randn(B, T, E, generator=g).to(torch.bfloat16).float()
d = torch.randn(B, T, E, generator=g).to(torch.bfloat16).float()
qv, dv = m(q.cuda(), d.cuda())
loss = tta.InfoNCELoss(compute_dtype=torch.bfloat16)(qv, dv)
loss.backward()
rl = cpu_ref.infonce(*cpu_ref.forward(q, d, p))
rl.backward()
print("loss", float(loss), float(rl))
for k, t in m.named_parameters():
    a, r = t.grad.double().cpu(), p[k].grad.double()
    print(f"{k:40s} frob {float((a - r).norm() / r.norm()):.4f} cos {float((a * r).sum() / (a.norm() * r.norm())):.5f}")
