"""Re-partition checkpoints to another tensor- or pipeline-parallel degree (reference
checkpoint/reshape_meg_2d.py, reshape_3d_utils.py, reshape_utils.py, deepspeed_checkpoint.py
``DeepSpeedCheckpoint``).

* Tensor parallel: an AutoTP checkpoint records, per sharded layer, its split dim and row layout
  (``tp_partitions``: contiguous, ("chunks", n) for packed gate|up, ("heads", counts, d) for packed
  GQA q|k|v) -- the TP=k model files are unsharded with module_inject.layers.unshard_rows and
  re-sharded to the new degree with shard_rows; replicated tensors are copied.
* Pipeline parallel: the pipeline engine stores one file per LAYER (``layer_XX-model_states.pt``),
  so any stage count can load them; reshaping writes the per-stage engine-state files for the new
  degree.
* Data parallel / ZeRO degree: the universal checkpoint (checkpoint/universal.py).

Everything is loaded with ``torch.load(weights_only=True)``.
"""
import glob
import os
import re
import shutil
from dataclasses import dataclass, field

import torch

from ..module_inject.layers import shard_rows, unshard_rows

_MP = re.compile(r"^mp_rank_(\d+)_model_states\.pt$")


def _load(path):
    return torch.load(path, map_location="cpu", weights_only=True)


def _layout(x):
    """Layouts round-trip through torch.save as lists; shard_rows expects tuples."""
    if x is None:
        return None
    return tuple(_layout(v) if isinstance(v, list) and v and isinstance(v[0], list) else v for v in x)


@dataclass
class CheckpointInfo:
    path: str
    tp_degree: int
    pp_degree: int
    dp_degree: int
    zero_stage: int
    layer_files: list = field(default_factory=list)
    model_files: list = field(default_factory=list)
    optim_files: list = field(default_factory=list)


def inspect_checkpoint(ckpt_dir, tag=None):
    """Degrees and files of a checkpoint tag directory (reference DeepSpeedCheckpoint :35)."""
    if tag is None and os.path.isfile(os.path.join(ckpt_dir, "latest")):
        with open(os.path.join(ckpt_dir, "latest")) as f:
            tag = f.read().strip()
    d = os.path.join(ckpt_dir, tag) if tag else ckpt_dir
    names = sorted(os.listdir(d))
    model = [n for n in names if _MP.match(n)]
    layers = [n for n in names if re.match(r"^layer_\d+", n)]
    optim = [n for n in names if n.endswith("_optim_states.pt")]
    z3 = [n for n in names if re.match(r"^zero_pp_rank_\d+_mp_rank_\d+_model_states\.pt$", n)]
    meta = _load(os.path.join(d, (model or z3)[0]))
    ds = meta.get("ds_config") or {}
    zs = int((ds.get("zero_optimization") or {}).get("stage", 0))
    pp = len(model) if layers else 1
    tp = int(meta.get("mp_world_size", 1)) if not layers else 1
    dp = int(meta.get("dp_world_size", 1))
    return CheckpointInfo(d, tp, pp, dp, zs, layers, model or z3, optim)


def reshape_tp_states(states, new_tp):
    """states: per-TP-rank model-state dicts (rank order) -> new_tp model-state dicts."""
    parts = states[0].get("tp_partitions") or {}
    old_tp = len(states)
    out = [dict(states[0]) for _ in range(new_tp)]
    mods = {}
    for key in states[0]["module"]:
        owner, _, leaf = key.rpartition(".")
        info = parts.get(owner)
        tensors = [sd["module"][key] for sd in states]
        if info is None or (leaf == "bias" and not info["bias_split"]):
            full, shards = tensors[0], None
        elif info["split_dim"] == 0:
            full = unshard_rows(tensors, _layout(info["layout"])) if old_tp > 1 else tensors[0]
            shards = [shard_rows(full, _layout(info["layout"]), new_tp, r) for r in range(new_tp)]
        else:
            full = torch.cat(tensors, dim=1) if old_tp > 1 else tensors[0]
            shards = list(full.chunk(new_tp, dim=1))
        for r in range(new_tp):
            mods.setdefault(r, {})[key] = (shards[r] if shards is not None else full).clone()
    for r in range(new_tp):
        out[r]["module"] = mods.get(r, {})
        out[r]["mp_world_size"] = new_tp
        if parts:
            out[r]["tp_partitions"] = parts
        out[r]["param_shapes"] = None  # rebuilt by the engine on load
    return out


def reshape_checkpoint(src_dir, dst_dir, new_tp=None, new_pp=None, tag=None):
    """Write a copy of checkpoint ``tag`` under ``dst_dir`` re-partitioned to ``new_tp`` (AutoTP
    model states) and/or ``new_pp`` (pipeline stage files). Optimizer partitions are not carried
    across a TP change (resume from the model states or convert through the universal format)."""
    info = inspect_checkpoint(src_dir, tag)
    tag = os.path.basename(info.path)
    out = os.path.join(dst_dir, tag)
    os.makedirs(out, exist_ok=True)
    if info.layer_files:  # pipeline checkpoint
        for n in info.layer_files:
            shutil.copyfile(os.path.join(info.path, n), os.path.join(out, n))
        stage0 = _load(os.path.join(info.path, info.model_files[0]))
        for s in range(new_pp or info.pp_degree):
            torch.save(dict(stage0), os.path.join(out, f"mp_rank_{s:02d}_model_states.pt"))
    else:
        states = [_load(os.path.join(info.path, n)) for n in info.model_files]
        new = reshape_tp_states(states, new_tp or info.tp_degree)
        for r, sd in enumerate(new):
            torch.save(sd, os.path.join(out, f"mp_rank_{r:02d}_model_states.pt"))
        if (new_tp or info.tp_degree) == info.tp_degree:
            for n in info.optim_files:
                shutil.copyfile(os.path.join(info.path, n), os.path.join(out, n))
    with open(os.path.join(dst_dir, "latest"), "w") as f:
        f.write(tag)
    return out


def tp_full_state_dict(ckpt_dir, tag=None):
    """Unsharded module state dict of an AutoTP checkpoint (reshape to TP=1)."""
    info = inspect_checkpoint(ckpt_dir, tag)
    states = [_load(os.path.join(info.path, n)) for n in info.model_files]
    return reshape_tp_states(states, 1)[0]["module"]


def pipeline_layer_files(ckpt_dir, tag=None):
    return sorted(glob.glob(os.path.join(inspect_checkpoint(ckpt_dir, tag).path, "layer_*-model_states.pt")))
