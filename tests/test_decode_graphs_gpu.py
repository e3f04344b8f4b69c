"""HIP-graph decode (inference/v2/decode_graphs.py): teacher-forced decode steps replayed from
captured graphs give the same logits as the eager ragged forward, across sequence / KV-length
buckets, with sequences joining and leaving between steps."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(model, graphs):
    from shuffle_exchange_amd.inference.v2 import RaggedInferenceEngineConfig, build_engine
    return build_engine(model, RaggedInferenceEngineConfig(kv_block_size=64, num_kv_blocks=128, decode_graphs=graphs))


def test_decode_graphs_match_eager():
    from shuffle_exchange_amd.models import LlamaForCausalLM, llama_config
    from shuffle_exchange_amd.ops import native
    native.require_hip()
    torch.manual_seed(0)
    cfg = llama_config("llama-tiny", hidden_size=512, intermediate_size=1024, num_attention_heads=4,
                       num_key_value_heads=2, vocab_size=512, num_hidden_layers=2,
                       max_position_embeddings=4096)
    model = LlamaForCausalLM(cfg).to("cuda", torch.bfloat16).eval()
    eg, ee = _engine(model, True), _engine(model, False)
    g = torch.Generator().manual_seed(1)
    lens = {0: 300, 1: 17, 2: 70}
    prompts = {u: torch.randint(0, 512, (n,), generator=g).tolist() for u, n in lens.items()}
    a = eg.put(list(prompts), list(prompts.values()))
    b = ee.put(list(prompts), list(prompts.values()))
    torch.testing.assert_close(a, b)  # prefill runs eagerly in both
    live = [0, 1, 2]
    for step in range(24):
        if step == 6:
            live = [0, 2]  # a sequence leaves: smaller bucket
        if step == 12:
            live = [0, 2, 3]  # a new sequence joins with a prefill, then decodes
            p = torch.randint(0, 512, (5,), generator=g).tolist()
            eg.put([3], [p])
            ee.put([3], [p])
        toks = [[int(torch.randint(0, 512, (1,), generator=g))] for _ in live]
        a = eg.put(live, toks)
        b = ee.put(live, toks)
        rel = ((a - b).norm() / b.norm()).item()
        assert rel < 2e-2, (step, rel)
    runner = eg._decode_runner()
    assert runner is not None and runner.replays == 24 and runner.num_graphs == 2  # (4, 512), (2, 512)
    assert ee._decode_runner() is None
    # KV-length bucket crossing: grow sequence 1 past 512 tokens (bucket 512 -> 1024)
    eg.put([1], [list(range(480))])
    ee.put([1], [list(range(480))])
    for _ in range(20):
        a = eg.put([1, 2], [[5], [6]])
        b = ee.put([1, 2], [[5], [6]])
        assert ((a - b).norm() / b.norm()).item() < 2e-2
    assert runner.num_graphs == 3  # + (2, 1024)
