import torch, math, sys
sys.path.insert(0, '.')
from shuffle_exchange_amd.ops import native
native.require_hip()
from shuffle_exchange_amd.ops.attention import reference_attention
torch.manual_seed(0)
B,S,H,D=1,128,1,128
def run(q,k,v,causal=False):
    o,lse=torch.ops.sxe.flash_attn_fwd(q,k,v,causal,1.0/math.sqrt(D))
    o2,lse2=reference_attention(q.float(),k.float(),v.float(),causal,1.0/math.sqrt(D),return_lse=True)
    return o.float(), o2.float(), lse, lse2
dev='cuda'
# probe 1: Q=0 -> uniform P; O = mean_k V
q=torch.zeros(B,S,H,D,device=dev,dtype=torch.bfloat16); k=torch.randn(B,S,H,D,device=dev,dtype=torch.bfloat16)
v=torch.randn(B,S,H,D,device=dev,dtype=torch.bfloat16)
o,o2,l,l2=run(q,k,v)
print("probe1 uniformP: maxerr", (o-o2).abs().max().item(), "lse err", (l-l2).abs().max().item())
print(" o[0,0,0,:8]", o[0,0,0,:8].tolist()); print(" ref", o2[0,0,0,:8].tolist())
print(" o[0,5,0,:8]", o[0,5,0,:8].tolist())
# probe 2: V = one-hot over d for key (d == key) -> O[q][d] = P[q][key=d]
v=torch.zeros(B,S,H,D,device=dev,dtype=torch.bfloat16)
for kk in range(S): v[0,kk,0,kk%D]=1.0
q=torch.randn(B,S,H,D,device=dev,dtype=torch.bfloat16)
o,o2,l,l2=run(q,k,v)
print("probe2 P-reveal: maxerr", (o-o2).abs().max().item(), "lse err", (l-l2).abs().max().item())
print(" o[0,0,0,:8]", [round(x,4) for x in o[0,0,0,:8].tolist()]); print(" ref", [round(x,4) for x in o2[0,0,0,:8].tolist()])
print(" o[0,1,0,:8]", [round(x,4) for x in o[0,1,0,:8].tolist()]); print(" ref", [round(x,4) for x in o2[0,1,0,:8].tolist()])
# probe 3: single key nonzero score
o,o2,l,l2=run(q,k,torch.randn_like(v))
print("probe3 random: maxerr", (o-o2).abs().max().item(), "lse err", (l-l2).abs().max().item())
