"""Flops profiler counts the analytic matmul FLOPs of a Llama forward and attributes them to
modules."""
import pytest
import torch


def test_llama_forward_flops():
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    from shuffle_exchange_amd.profiling.flops_profiler import FlopsProfiler, get_model_profile
    m = LlamaForCausalLM(llama_config("llama-tiny"))
    ids = torch.randint(0, 512, (2, 64))
    flops, macs, params = get_model_profile(m, args=[ids], print_profile=False, as_string=False)
    T = ids.numel()
    lin = sum(p.numel() for n, p in m.named_parameters() if n.endswith("proj.weight"))
    head = m.lm_head.weight.numel()
    assert flops >= 2 * T * (lin + head)  # attention score/value matmuls come on top
    assert macs == flops / 2 and params == sum(p.numel() for p in m.parameters())
    prof = FlopsProfiler(m)
    prof.start_profile()
    m(ids)
    prof.stop_profile()
    rows = {name: fl for name, d, p, fl, lat in prof.module_profile()}
    assert rows["lm_head"] == 2 * T * head
    text = prof.print_model_profile(module_depth=1, detailed=False, output_file=None)
    assert "fwd FLOPs" in text


def test_conv_and_attention_counted():
    """Convolutions and SDPA attention are counted at the ATen level (reference counts conv /
    matmul / softmax-context via its functional patches)."""
    import torch.nn as nn
    import torch.nn.functional as F
    from shuffle_exchange_amd.profiling.flops_profiler import FlopsProfiler

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = nn.Conv2d(3, 8, 3, padding=1, bias=False)

        def forward(self, x, q, k, v):
            return self.conv(x), F.scaled_dot_product_attention(q, k, v)

    m = M()
    x = torch.randn(2, 3, 16, 16)
    q = k = v = torch.randn(2, 4, 32, 16)
    prof = FlopsProfiler(m)
    prof.start_profile()
    m(x, q, k, v)
    prof.stop_profile()
    conv = 2 * 2 * 8 * 16 * 16 * 3 * 3 * 3
    attn = 2 * (2 * 2 * 4 * 32 * 32 * 16)  # QK^T and PV
    assert prof.get_total_flops() == conv + attn
    assert dict((n, f) for n, d, p, f, lat in prof.module_profile())["conv"] == conv


@pytest.mark.gpu
def test_hip_ops_have_flop_formulas():
    """The hand-written gfx950 GEMMs (skinny decode GEMM, grouped expert GEMM, k-major wgrad) and
    flash attention are counted on the GPU, not silently dropped."""
    from shuffle_exchange_amd.ops import native
    from torch.utils.flop_counter import FlopCounterMode
    from shuffle_exchange_amd.profiling.flops_profiler.profiler import _register_sxe_formulas
    native.require_hip()
    _register_sxe_formulas()
    dev, bf = "cuda", torch.bfloat16
    x, w = torch.randn(2, 256, device=dev, dtype=bf), torch.randn(512, 256, device=dev, dtype=bf)
    xs, we = torch.randn(300, 256, device=dev, dtype=bf), torch.randn(4, 384, 256, device=dev, dtype=bf)
    offs = torch.tensor([0, 100, 100, 250, 300], dtype=torch.int32, device=dev)
    a, b = torch.randn(256, 512, device=dev, dtype=bf), torch.randn(256, 768, device=dev, dtype=bf)
    c = torch.zeros(512, 768, device=dev)
    q = torch.randn(1, 128, 2, 128, device=dev, dtype=bf)
    with FlopCounterMode(display=False) as fc:
        torch.ops.sxe.skinny_gemm(x, w, None)
        torch.ops.sxe.grouped_gemm(xs, we, offs, None)
        torch.ops.sxe.wgrad_gemm_(a, b, c, 1.0, False)
        torch.ops.sxe.flash_attn_fwd(q, q, q, True, 0.088)
    expect = 2 * 2 * 512 * 256 + 2 * 300 * 384 * 256 + 2 * 256 * 512 * 768 + 4 * 2 * 128 * 128 * 128 // 2
    assert fc.get_total_flops() == expect
