"""FastFileWriter (reference io/fast_file_writer.py): torch.save through pinned double buffers into the
C++ AIO engine yields a byte-identical file; the fast checkpoint engine round-trips an engine."""
import io

import torch

from . import _dist_cases as C
from .dist_utils import run_dist


def test_fast_file_writer_matches_torch_save(tmp_path):
    from shuffle_exchange_amd.io import FastFileWriter, FastFileWriterConfig, MockFileWriter
    sd = {"a": torch.randn(300_000), "b": torch.arange(12345, dtype=torch.int32), "c": {"d": torch.ones(7, 3)}}
    ref = io.BytesIO()
    torch.save(sd, ref)
    p = str(tmp_path / "x.pt")
    w = FastFileWriter(p, FastFileWriterConfig(buffer_size=64 << 10))  # many buffer swaps + an unaligned tail
    torch.save(sd, w)
    w.close()
    assert open(p, "rb").read() == ref.getvalue()
    assert w._get_file_stats()["aio_writes"] > 2
    back = torch.load(p, weights_only=True)
    assert torch.equal(back["a"], sd["a"]) and torch.equal(back["c"]["d"], sd["c"]["d"])
    m = MockFileWriter()
    torch.save(sd, m)
    assert m.num_bytes == len(ref.getvalue())


def _case(rank, world, tmpdir):
    import shuffle_exchange_amd as sxe
    model, cfg = C.tiny_llama(0)
    ds = {"train_micro_batch_size_per_gpu": 1, "zero_optimization": {"stage": 2},
          "checkpoint": {"writer": {"type": "fast", "io_buffer_size": 1 << 20}},
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}}
    eng, _, _, _ = sxe.initialize(model=model, config=ds)
    b = C.global_batches(cfg, world, 1, 16, 1)[0][rank:rank + 1]
    loss = eng(b, labels=b)
    eng.backward(loss)
    eng.step()
    eng.save_checkpoint(tmpdir, tag="t1")
    before = C.full_params(eng)
    model2, _ = C.tiny_llama(1)
    eng2, _, _, _ = sxe.initialize(model=model2, config=ds)
    eng2.load_checkpoint(tmpdir, tag="t1")
    after = C.full_params(eng2)
    return {"kind": type(eng.checkpoint_engine).__name__,
            "same": all(torch.equal(before[k], after[k]) for k in before)}


def test_fast_checkpoint_engine_roundtrip(tmp_path):
    for r in run_dist(_case, 2, str(tmp_path)):
        assert r["kind"] == "FastCheckpointEngine" and r["same"]
