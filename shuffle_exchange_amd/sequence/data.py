"""Sequence-parallel data sharding (parity: reference runtime/sequence_parallel/ulysses_sp.py:426-552
``UlyssesSPDataLoaderAdapter``).

Labels are shifted over the FULL sequence before sharding (the last token of chunk r predicts the
first token of chunk r+1), then input ids, shifted labels and global position ids are cut into
``sp_size`` contiguous chunks; rank r of the SP group gets chunk r."""
import torch


def shard_batch_for_sp(input_ids, sp_rank, sp_size, labels=None, ignore_index=-100):
    B, S = input_ids.shape
    assert S % sp_size == 0, f"sequence length {S} must be divisible by sp_size {sp_size}"
    labels = input_ids if labels is None else labels
    shifted = torch.cat([labels[:, 1:], torch.full_like(labels[:, :1], ignore_index)], dim=1)
    c = S // sp_size
    sl = slice(sp_rank * c, (sp_rank + 1) * c)
    pos = torch.arange(S, device=input_ids.device)[sl].unsqueeze(0).expand(B, c)
    return {"input_ids": input_ids[:, sl].contiguous(), "labels": shifted[:, sl].contiguous(),
            "position_ids": pos.contiguous(), "shift_labels": False}


class UlyssesSPDataLoaderAdapter:
    """Wraps an iterable of full-sequence batches (tensor or dict with ``input_ids``/``labels``)."""

    def __init__(self, dl, sp_rank, sp_world_size, device=None, ignore_index=-100):
        self.dl = dl
        self.sp_rank, self.sp_world_size = sp_rank, sp_world_size
        self.device = device
        self.ignore_index = ignore_index

    def __len__(self):
        return len(self.dl)

    def __iter__(self):
        for batch in self.dl:
            if isinstance(batch, dict):
                ids, labels = batch["input_ids"], batch.get("labels")
            else:
                ids, labels = batch, None
            if self.device is not None:
                ids = ids.to(self.device)
                labels = labels.to(self.device) if labels is not None else None
            yield shard_batch_for_sp(ids, self.sp_rank, self.sp_world_size, labels, self.ignore_index)
