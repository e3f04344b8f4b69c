"""Data pipeline: Megatron-format mmap indexed dataset (byte layout, builder, merge, zero-copy
reads) and token-budget variable batch size with per-batch LR scaling."""
import struct

import numpy as np
import torch


def test_mmap_indexed_dataset_roundtrip_and_format(tmp_path):
    from shuffle_exchange_amd.runtime.data_pipeline.indexed_dataset import (MMapIndexedDataset, data_file_path,
                                                                            index_file_path, make_builder)
    rng = np.random.default_rng(0)
    docs = [[rng.integers(0, 50000, size=rng.integers(1, 40)) for _ in range(rng.integers(1, 4))] for _ in range(20)]
    prefix = str(tmp_path / "corpus")
    b = make_builder(data_file_path(prefix), vocab_size=50000)
    for d in docs:
        for s in d:
            b.add_item(torch.from_numpy(s.astype(np.int64)))
        b.end_document()
    b.finalize(index_file_path(prefix))
    ds = MMapIndexedDataset(prefix)
    items = [s for d in docs for s in d]
    assert len(ds) == len(items) and ds.dtype == np.uint16
    for i, s in enumerate(items):
        assert np.array_equal(ds[i], s)
    assert np.array_equal(ds.get(3, offset=1, length=1), items[3][1:2]) or len(items[3]) < 2
    assert ds.doc_idx[-1] == len(items) and len(ds.doc_idx) == len(docs) + 1
    # header bytes (reference indexed_dataset.py:371-404)
    raw = open(index_file_path(prefix), "rb").read()
    assert raw[:9] == b"MMIDIDX\x00\x00" and struct.unpack("<Q", raw[9:17]) == (1,) and raw[17] == 6
    # merge
    b2 = make_builder(str(tmp_path / "m.bin"), vocab_size=50000)
    b2.merge_file_(prefix)
    b2.merge_file_(prefix)
    b2.finalize(str(tmp_path / "m.idx"))
    m = MMapIndexedDataset(str(tmp_path / "m"))
    assert len(m) == 2 * len(items) and np.array_equal(m[len(items) + 5], items[5])


def test_variable_batch_size_and_lr():
    from shuffle_exchange_amd.runtime.data_pipeline.variable_batch_size_and_lr import (
        batch_by_seqlens, get_dataloader_and_lr_scheduler_for_variable_batch_size, scale_lr)
    rng = np.random.default_rng(1)
    seqlens = rng.integers(4, 60, size=200).tolist()
    mbs, sizes, mx = batch_by_seqlens(seqlens, max_tokens=128, effective_batch_size=4, sequence_picking_order="seqlen")
    for b, ids in mbs:
        assert sum(seqlens[i] for i in ids) <= 128
    assert len(mbs) == 4 * len(sizes) and all(s > 0 for s in sizes)
    seen = [i for _, ids in mbs for i in ids]
    assert len(seen) == len(set(seen))
    assert scale_lr(8, 16, 1.0, "linear") == 2.0 and abs(scale_lr(8, 32, 1.0, "sqrt") - 2.0) < 1e-12

    data = [torch.arange(n) for n in seqlens]
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=0.1)
    dl, sched = get_dataloader_and_lr_scheduler_for_variable_batch_size(
        data, seqlens, max_tokens=128, effective_batch_size=2, lr_scheduler_or_optimizer=opt,
        dataloader_rank=1, dataloader_num_replicas=2, base_batch_size=4, lr_scaling_method="linear",
        sequence_picking_order="random", seed=0)
    first = next(iter(dl))
    assert isinstance(first, list) and sum(len(s) for s in first) <= 128
    lrs = []
    for _ in range(3):
        lrs.append(opt.param_groups[0]["lr"])
        sched.step()
    _, sizes2, _ = batch_by_seqlens(seqlens, 128, effective_batch_size=2, sequence_picking_order="random", seed=0)
    assert np.allclose(lrs, [0.1 * s / 4 for s in sizes2[:3]])
