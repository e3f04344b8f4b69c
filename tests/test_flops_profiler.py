"""Flops profiler counts the analytic matmul FLOPs of a Llama forward and attributes them to
modules."""
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
