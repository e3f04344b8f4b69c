"""Variable batch size by token budget, with the learning rate scaled per batch.

Parity: reference runtime/data_pipeline/data_sampling/variable_batch_size_and_lr.py --
``batch_by_seqlens`` :23 (pack samples into micro-batches whose summed sequence length stays under
``max_tokens``; picking order dataloader / random / seqlen; micro-batches grouped into batches of
``effective_batch_size`` = gradient-accumulation x data-parallel), ``scale_lr`` :149 (linear / sqrt),
``dataloader_for_variable_batch_size`` :165, ``VariableBatchSizeLR`` :226,
``lr_scheduler_for_variable_batch_size`` :308 and
``get_dataloader_and_lr_scheduler_for_variable_batch_size`` :432.

The packer here is a single greedy pass (O(n)) instead of the reference's search over batch ends:
on MI355X the point of token-budget batching is to keep every micro-batch's GEMMs the same size
(tokens per micro-batch ~ max_tokens), which the greedy fill achieves.
"""
import math
import random

import numpy as np
import torch

from ...utils.logging import logger


def batch_by_seqlens(seqlens, max_tokens, sequence_ids_per_mb=None, min_batch_size=1, max_batch_size=None,
                     sequence_picking_order="dataloader", effective_batch_size=1,
                     required_microbatches_of_same_size=False, verbose=False, seed=None):
    """Returns (microbatch_ids: [(batch_id, [sample ids])], batch_sizes: samples per batch,
    batch_max_seqlens: longest sample per batch)."""
    assert sequence_picking_order in ("random", "seqlen", "dataloader")
    ids = list(range(len(seqlens))) if sequence_ids_per_mb is None else list(sequence_ids_per_mb)
    metrics = [(int(seqlens[i]), i) for i in ids]
    if sequence_picking_order == "random":
        random.Random(seed).shuffle(metrics)
    elif sequence_picking_order == "seqlen":
        metrics.sort()
    too_long = [i for v, i in metrics if v > max_tokens]
    if too_long:
        logger.warning(f"samples {too_long[:8]}{'...' if len(too_long) > 8 else ''} exceed max_tokens={max_tokens}; "
                       f"dropped")
        metrics = [(v, i) for v, i in metrics if v <= max_tokens]
    mbs, cur, cur_tok = [], [], 0
    for v, i in metrics:
        if cur and (cur_tok + v > max_tokens or (max_batch_size and len(cur) >= max_batch_size)):
            mbs.append(cur)
            cur, cur_tok = [], 0
        cur.append((v, i))
        cur_tok += v
    if cur and len(cur) >= (min_batch_size or 1):
        mbs.append(cur)
    mbs = [m for m in mbs if len(m) >= (min_batch_size or 1)]
    E = max(1, int(effective_batch_size))
    n_batches = len(mbs) // E
    if len(mbs) % E:
        logger.info(f"dropping {len(mbs) % E} trailing micro-batches that do not fill a batch of {E}")
    if required_microbatches_of_same_size:
        # trim every micro-batch of a batch to the batch's smallest micro-batch size
        for b in range(n_batches):
            grp = mbs[b * E:(b + 1) * E]
            k = min(len(m) for m in grp)
            for j in range(E):
                mbs[b * E + j] = grp[j][:k]
    microbatch_ids, batch_sizes, batch_max = [], [], []
    for b in range(n_batches):
        grp = mbs[b * E:(b + 1) * E]
        for m in grp:
            microbatch_ids.append((b, [i for _, i in m]))
        batch_sizes.append(sum(len(m) for m in grp))
        batch_max.append(max(v for m in grp for v, _ in m))
    if verbose:
        logger.info(f"variable batching: {len(microbatch_ids)} micro-batches in {n_batches} batches, "
                    f"samples/batch min {min(batch_sizes, default=0)} max {max(batch_sizes, default=0)}")
    return microbatch_ids, batch_sizes, batch_max


def scale_lr(base_batch_size, batch_size, base_lr=1, method="linear"):
    if method == "linear":
        return base_lr * batch_size / base_batch_size
    if method == "sqrt":
        return base_lr * math.sqrt(batch_size / base_batch_size)
    if method is None or method.upper() == "NONE":
        return base_lr
    raise ValueError(f"unknown lr scaling method {method}")


def dataloader_for_variable_batch_size(dataset, microbatch_ids, batch_max_seqlens, dataloader_rank=0,
                                       dataloader_batch_size=1, dataloader_num_replicas=1, dataloader_collate_fn=None,
                                       dataloader_num_workers=2, dataloader_pin_memory=False,
                                       required_microbatches_of_same_seqlen=False, sample_padding_fn=None):
    """Loader over this data-parallel rank's micro-batches (micro-batch j of every batch goes to rank
    j % replicas). Each item is the list of samples of one micro-batch, optionally padded to the
    batch's max length (``required_microbatches_of_same_seqlen``) through ``sample_padding_fn``."""
    mine = [(b, ids) for k, (b, ids) in enumerate(microbatch_ids) if k % dataloader_num_replicas == dataloader_rank]

    def collate(items):
        (b, ids), = items
        samples = [dataset[i] for i in ids]
        if required_microbatches_of_same_seqlen and sample_padding_fn is not None:
            samples = [sample_padding_fn(s, batch_max_seqlens[b]) for s in samples]
        return dataloader_collate_fn(samples) if dataloader_collate_fn is not None else samples

    return torch.utils.data.DataLoader(mine, batch_size=1, shuffle=False, collate_fn=collate,
                                       num_workers=dataloader_num_workers, pin_memory=dataloader_pin_memory)


class VariableBatchSizeLR:
    """Scales the wrapped scheduler's learning rate by the size of the batch being stepped."""

    def __init__(self, lr_scheduler, base_batch_size, batch_sizes, dataloader=None, lr_scaling_method="linear"):
        self.base_lr_scheduler = lr_scheduler
        self.base_batch_size, self.batch_sizes = base_batch_size, list(batch_sizes)
        self.dataloader, self.method = dataloader, lr_scaling_method
        self.last_epoch = -1
        self.step()

    @property
    def optimizer(self):
        return self.base_lr_scheduler.optimizer

    def state_dict(self):
        return {"base_lr_scheduler": self.base_lr_scheduler.state_dict(), "base_batch_size": self.base_batch_size,
                "batch_sizes": self.batch_sizes, "lr_scaling_method": self.method, "last_epoch": self.last_epoch}

    def load_state_dict(self, sd):
        self.base_lr_scheduler.load_state_dict(sd["base_lr_scheduler"])
        self.base_batch_size, self.batch_sizes = sd["base_batch_size"], sd["batch_sizes"]
        self.method, self.last_epoch = sd["lr_scaling_method"], sd["last_epoch"]

    def get_last_lr(self):
        return self._last_lr

    def get_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups]

    def step(self, epoch=None):
        if self.last_epoch >= 0:  # undo the previous scaling before the base scheduler steps
            for g, base in zip(self.optimizer.param_groups, self._unscaled):
                g["lr"] = base
            self.base_lr_scheduler.step()
        self.last_epoch += 1
        bs = self.batch_sizes[min(self.last_epoch, len(self.batch_sizes) - 1)] if self.batch_sizes else \
            self.base_batch_size
        self._unscaled = [g["lr"] for g in self.optimizer.param_groups]
        for g in self.optimizer.param_groups:
            g["lr"] = scale_lr(self.base_batch_size, bs, g["lr"], self.method)
        self._last_lr = [g["lr"] for g in self.optimizer.param_groups]


def lr_scheduler_for_variable_batch_size(base_batch_size, batch_sizes, dataloader, lr_scheduler_or_optimizer,
                                         lr_scaling_method="linear"):
    sched = lr_scheduler_or_optimizer
    if isinstance(sched, torch.optim.Optimizer) or not hasattr(sched, "step") or not hasattr(sched, "optimizer"):
        sched = torch.optim.lr_scheduler.LambdaLR(lr_scheduler_or_optimizer, lambda _: 1.0)
    return VariableBatchSizeLR(sched, base_batch_size, batch_sizes, dataloader, lr_scaling_method)


def get_dataloader_and_lr_scheduler_for_variable_batch_size(dataset, dataset_seqlens, max_tokens,
                                                            effective_batch_size, lr_scheduler_or_optimizer,
                                                            sequence_picking_order="dataloader",
                                                            dataloader_rank=0, dataloader_num_replicas=1,
                                                            dataloader_collate_fn=None, dataloader_num_workers=0,
                                                            base_batch_size=1, lr_scaling_method="linear",
                                                            min_batch_size=1, max_batch_size=None, seed=None,
                                                            required_microbatches_of_same_size=False,
                                                            required_microbatches_of_same_seqlen=False,
                                                            sample_padding_fn=None, verbose=False):
    mb_ids, batch_sizes, batch_max = batch_by_seqlens(
        np.asarray(dataset_seqlens), max_tokens, min_batch_size=min_batch_size, max_batch_size=max_batch_size,
        sequence_picking_order=sequence_picking_order, effective_batch_size=effective_batch_size,
        required_microbatches_of_same_size=required_microbatches_of_same_size, verbose=verbose, seed=seed)
    dl = dataloader_for_variable_batch_size(dataset, mb_ids, batch_max, dataloader_rank,
                                            dataloader_num_replicas=dataloader_num_replicas,
                                            dataloader_collate_fn=dataloader_collate_fn,
                                            dataloader_num_workers=dataloader_num_workers,
                                            required_microbatches_of_same_seqlen=required_microbatches_of_same_seqlen,
                                            sample_padding_fn=sample_padding_fn)
    sched = lr_scheduler_for_variable_batch_size(base_batch_size, batch_sizes, dl, lr_scheduler_or_optimizer,
                                                 lr_scaling_method)
    return dl, sched
