"""Compression: QAT linears with STE, scheduled pruning masks, row pruning that physically shrinks
the layer and its consumer, layer reduction."""
import torch
import torch.nn as nn


class MLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.layers = nn.ModuleList([nn.Sequential() for _ in range(4)])
        self.fc1 = nn.Linear(16, 32)
        self.fc2 = nn.Linear(32, 16)

    def forward(self, x):
        return self.fc2(torch.relu(self.fc1(x)))


CFG = {"compression_training": {
    "weight_quantization": {"shared_parameters": {"enabled": True, "schedule_offset": 0, "quantize_groups": 1},
                            "different_groups": {"wq": {"params": {"start_bits": 8, "target_bits": 4,
                                                                   "quantization_period": 1}, "modules": ["fc2"]}}},
    "sparse_pruning": {"shared_parameters": {"enabled": True, "schedule_offset": 2, "method": "l1"},
                       "different_groups": {"sp": {"params": {"dense_ratio": 0.25}, "modules": ["fc2"]}}},
    "row_pruning": {"shared_parameters": {"enabled": True, "schedule_offset": 0},
                    "different_groups": {"rp": {"params": {"dense_ratio": 0.5}, "modules": ["fc1"],
                                                "related_modules": [["fc2"]]}}},
    "layer_reduction": {"enabled": True, "keep_number_layer": 2, "module_name_prefix": "layers",
                        "teacher_layer": [1, 3]}}}


def test_compression_pipeline():
    from shuffle_exchange_amd.compression import (LinearLayer_Compress, compression_scheduler, init_compression,
                                                  redundancy_clean)
    torch.manual_seed(0)
    m = init_compression(MLP(), CFG)
    assert len(m.layers) == 2 and isinstance(m.fc1, LinearLayer_Compress) and isinstance(m.fc2, LinearLayer_Compress)
    sch = compression_scheduler(m, CFG)
    opt = torch.optim.SGD(m.parameters(), lr=0.01)
    x = torch.randn(8, 16)
    for _ in range(4):
        sch.step()
        loss = m(x).pow(2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
    assert m.fc2.weight.grad is not None  # STE lets grads through the quantizer
    assert m.fc2.sparse_pruning_enabled and m.fc2.wq["bits"] == 4
    out_before = m(x)
    redundancy_clean(m, CFG)
    assert m.fc1.weight.shape == (16, 16) and m.fc2.weight.shape == (16, 16)
    assert torch.allclose(m(x), out_before, atol=1e-5)
    assert (m.fc2.weight == 0).float().mean() >= 0.7
