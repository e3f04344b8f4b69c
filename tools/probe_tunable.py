"""Print this box's TunableOp validators (to compare with the packaged table header)."""
import torch
torch.cuda.tunable.enable(True)
torch.cuda.tunable.tuning_enable(False)
a = torch.randn(256, 256, device="cuda", dtype=torch.bfloat16)
(a @ a).sum().item()
for k, v in torch.cuda.tunable.get_validators():
    print("Validator", k, v)
