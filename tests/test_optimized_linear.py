"""OptimizedLinear / LoRA: only LoRA weights train, output = base + alpha/r * B A x, FP8-quantized
base is close to the bf16 base, sharded base weight gathers back to the full weight (gloo)."""
import torch

from .dist_utils import run_dist


def test_lora_linear_forward_and_grads():
    from shuffle_exchange_amd.linear import LoRAConfig, OptimizedLinear
    torch.manual_seed(0)
    lin = OptimizedLinear(32, 48, lora_config=LoRAConfig(lora_r=4, lora_alpha=8), dtype=torch.float32)
    x = torch.randn(5, 32)
    y0 = lin(x)
    assert torch.allclose(y0, x @ lin.base_weight.t(), atol=1e-5)  # B starts at zero
    with torch.no_grad():
        lin.lora_weight_2.normal_()
    y = lin(x)
    ref = x @ lin.base_weight.t() + 2.0 * (x @ lin.lora_weight_1.t()) @ lin.lora_weight_2.t()
    assert torch.allclose(y, ref, atol=1e-4)
    y.sum().backward()
    assert lin.base_weight.grad is None and lin.lora_weight_1.grad is not None


def test_quantized_base():
    from shuffle_exchange_amd.linear import LoRAConfig, OptimizedLinear, QuantizationConfig
    torch.manual_seed(0)
    lin = OptimizedLinear(256, 128, lora_config=LoRAConfig(lora_r=2), quantization_config=QuantizationConfig(
        group_size=128), dtype=torch.float32)
    full = lin.full_weight().float()
    assert full.shape == (128, 256)
    x = torch.randn(3, 256)
    assert torch.isfinite(lin(x)).all()


def _case_sharded(rank, world):
    from shuffle_exchange_amd.linear import LoRAConfig, OptimizedLinear
    torch.manual_seed(0)
    w = torch.randn(64, 16)
    lin = OptimizedLinear(16, 64, lora_config=LoRAConfig(lora_r=2, base_weight_sharding=world), dtype=torch.float32)
    lin.load_base_weight(w)
    return {"local_rows": lin.base_weight.shape[0], "ok": bool(torch.equal(lin.full_weight(), w))}


def test_sharded_base_weight():
    for r in run_dist(_case_sharded, 2):
        assert r["local_rows"] == 32 and r["ok"]
