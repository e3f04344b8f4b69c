"""Post-training group-wise weight quantization (reference inference/quantization): replaced
modules keep the model's outputs within the quantization error, memory shrinks, int4 packs 2/byte."""
import pytest
import torch


@pytest.mark.parametrize("bits,sym,tol", [(8, False, 2e-2), (4, False, 2e-1), (8, True, 2e-2), (4, True, 3e-1)])
def test_quantized_linear_and_embedding(bits, sym, tol):
    from shuffle_exchange_amd.inference.quantization import QuantizedEmbedding, QuantizedLinear, quantize_model
    torch.manual_seed(0)
    model = torch.nn.Sequential()
    model.add_module("emb", torch.nn.Embedding(64, 128))
    model.add_module("fc1", torch.nn.Linear(128, 256))
    model.add_module("act", torch.nn.GELU())
    model.add_module("fc2", torch.nn.Linear(256, 64))
    ids = torch.randint(0, 64, (4, 8))
    ref = model(ids)
    cfg = {"num_bits": bits, "group_size": 64, "symmetric": sym}
    quantize_model(model, {"fc": cfg, "emb": cfg})
    assert isinstance(model.fc1, QuantizedLinear) and isinstance(model.emb, QuantizedEmbedding)
    assert model._sxe_quantized_modules == 3
    out = model(ids)
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < tol, rel
    nbytes = model.fc1.qweight.q.numel()
    assert nbytes == 128 * 256 * bits // 8
