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


class ConvNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(10, 4)
        self.conv1 = nn.Conv2d(4, 16, 3, padding=1)
        self.bn1 = nn.BatchNorm2d(16)
        self.conv2 = nn.Conv2d(16, 8, 3, padding=1)

    def forward(self, ids):
        x = self.emb(ids).permute(0, 3, 1, 2)  # [B, 4, H, W]
        return self.conv2(torch.relu(self.bn1(self.conv1(x))))


CONV_CFG = {"compression_training": {
    "weight_quantization": {"shared_parameters": {"enabled": True, "schedule_offset": 0, "quantize_groups": 1},
                            "different_groups": {"wq": {"params": {"start_bits": 8, "target_bits": 8,
                                                                   "quantization_period": 1},
                                                        "modules": ["emb", "conv2"]}}},
    "channel_pruning": {"shared_parameters": {"enabled": True, "schedule_offset": 1, "method": "l1"},
                        "different_groups": {"cp": {"params": {"dense_ratio": 0.5}, "modules": ["conv1"],
                                                    "related_modules": [["bn1", "conv2"]]}}}}}


def test_conv_channel_pruning_and_embedding_quantization():
    """Conv2d / BatchNorm / Embedding layers (reference basic_layer.py Conv2dLayer_Compress,
    BNLayer_Compress, Embedding_Compress): channel pruning masks conv1's weakest filters, then
    redundancy_clean physically drops them from conv1, bn1 and conv2's input channels with the
    output unchanged."""
    from shuffle_exchange_amd.compression import (BNLayer_Compress, Conv2dLayer_Compress, Embedding_Compress,
                                                  compression_scheduler, init_compression, redundancy_clean)
    torch.manual_seed(0)
    m = init_compression(ConvNet(), CONV_CFG)
    assert isinstance(m.conv1, Conv2dLayer_Compress) and isinstance(m.conv2, Conv2dLayer_Compress)
    assert isinstance(m.bn1, BNLayer_Compress) and isinstance(m.emb, Embedding_Compress)
    sch = compression_scheduler(m, CONV_CFG)
    opt = torch.optim.SGD(m.parameters(), lr=0.01)
    ids = torch.randint(0, 10, (2, 6, 6))
    for _ in range(3):
        sch.step()
        loss = m(ids).pow(2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
    assert m.conv1.channel_pruning_enabled and m.emb.weight_quantization_enabled
    assert int(m.conv1.channel_mask.sum()) == 8
    m.eval()
    before = m(ids)
    redundancy_clean(m, CONV_CFG)
    assert m.conv1.weight.shape[0] == 8 and m.conv1.out_channels == 8 and m.bn1.num_features == 8
    assert m.bn1.running_mean.shape == (8,) and m.conv2.weight.shape[1] == 8 and m.conv2.in_channels == 8
    torch.testing.assert_close(m(ids), before, atol=1e-5, rtol=1e-5)
    # the 8-bit fake quantization is baked into the embedding: at most 2^8 levels per group
    assert m.emb.weight.unique().numel() <= 256 and not m.emb.weight_quantization_enabled
