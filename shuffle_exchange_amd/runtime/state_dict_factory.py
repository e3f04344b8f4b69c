"""Model-weight loading for inference and ``load_module_only``: one entry point for every checkpoint
form, merged / split to the tensor-parallel degree of the running job.

Parity: reference runtime/state_dict_factory.py:21 ``SDLoaderFactory`` (``get_sd_loader_json``: the
JSON descriptor {"type", "checkpoints", "version", "parallelization", "mp_size"}), ``MegatronSDLoader``
merge/split of ``mp_rank_*`` shards (:190-420), and inference/engine.py:411-468 ``_load_checkpoint``.

Accepted sources (``load_state_dict_source``):
* a file: ``torch.save`` state dict (or a training model-states dict with ``module``), or
  ``*.safetensors``;
* a JSON descriptor (path or dict): ``checkpoints`` is the list of per-MP-rank files (relative to the
  descriptor's directory or ``base_dir``), optionally a ``tp_partitions`` map;
* a training checkpoint directory (``latest`` file or a tag directory) holding
  ``mp_rank_XX_model_states.pt`` (AutoTP ranks) or ZeRO-3 ``zero_pp_rank_*`` files with the
  consolidated 16-bit module.

MP merge: shards are unsharded to the full model with the recorded ``tp_partitions`` layouts
(checkpoint/reshape.py: packed q|k|v heads, gate|up chunks) when the checkpoint has them; otherwise
each tensor is matched against the target model's full shape -- equal shapes are replicated, a shape
whose one differing dim sums to the full dim is concatenated along it. The merged dict then loads
into the UNSHARDED model (strict by default: a missing or unexpected key raises with the key list),
and the job's own TP sharding (AutoTP / injected-layer slicing) splits it to the running degree --
merge and split are one path. Everything is read with ``weights_only=True`` / safetensors.
"""
import json
import os
import re

import torch

_MP = re.compile(r"^mp_rank_(\d+)_model_states\.pt$")


def _load_file(path):
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path, device="cpu")
    return torch.load(path, map_location="cpu", weights_only=True)


def _module_of(sd):
    if isinstance(sd, dict) and isinstance(sd.get("module"), dict):
        return sd["module"], sd
    if isinstance(sd, dict) and isinstance(sd.get("model"), dict):
        return sd["model"], sd
    return sd, {}


def _descriptor_files(desc, base):
    files = desc.get("checkpoints") or desc.get("checkpoint") or []
    if isinstance(files, str):
        files = [files]
    if isinstance(files, dict):  # {"non_tp": [...], "tp": [...]} (reference BLOOM descriptors): TP shards
        files = list(files.get("tp", [])) or list(files.get("non_tp", []))
    base = desc.get("base_dir", base)
    return [f if os.path.isabs(f) else os.path.join(base, f) for f in files]


def read_shards(source):
    """(list of per-MP-rank module state dicts, metadata dict) of a checkpoint source."""
    meta = {}
    if isinstance(source, dict):
        files = _descriptor_files(source, os.getcwd())
        meta.update({k: v for k, v in source.items() if k != "checkpoints"})
    elif isinstance(source, str) and source.endswith(".json") and os.path.isfile(source):
        with open(source) as f:
            desc = json.load(f)
        files = _descriptor_files(desc, os.path.dirname(os.path.abspath(source)))
        meta.update({k: v for k, v in desc.items() if k != "checkpoints"})
    elif isinstance(source, str) and os.path.isdir(source):
        d = source
        if os.path.isfile(os.path.join(d, "latest")):
            with open(os.path.join(d, "latest")) as f:
                d = os.path.join(d, f.read().strip())
        names = sorted(os.listdir(d))
        mp = sorted((n for n in names if _MP.match(n)), key=lambda n: int(_MP.match(n).group(1)))
        if not mp:  # ZeRO-3: the consolidated module lives in the zero_pp_rank files
            mp = [n for n in names if re.match(r"^zero_pp_rank_0_mp_rank_\d+_model_states\.pt$", n)]
        if not mp:
            hf = [n for n in names if n.endswith(".safetensors") or n in ("pytorch_model.bin", "model.pt")]
            mp = hf
        if not mp:
            raise FileNotFoundError(f"no model-state files (mp_rank_*_model_states.pt, *.safetensors) under {d}")
        files = [os.path.join(d, n) for n in mp]
        if all(n.endswith(".safetensors") for n in mp) and len(mp) > 1:  # HF sharded safetensors: one model
            merged = {}
            for f in files:
                merged.update(_load_file(f))
            return [merged], meta
    elif isinstance(source, str):
        files = [source]
    else:
        raise TypeError(f"checkpoint source must be a path or a descriptor dict, got {type(source).__name__}")
    if not files:
        raise ValueError(f"checkpoint descriptor {source!r} lists no files")
    shards = []
    for f in files:
        mod, full = _module_of(_load_file(f))
        if mod is None:
            raise ValueError(f"{f}: no module weights in this file (ZeRO-3 checkpoints need "
                             f"stage3_gather_16bit_weights_on_model_save=True to carry them)")
        if full.get("tp_partitions") and "tp_partitions" not in meta:
            meta["tp_partitions"] = full["tp_partitions"]
        shards.append(mod)
    return shards, meta


def merge_shards(shards, full_shapes=None, meta=None):
    """Full state dict from per-MP-rank shards (see the module docstring for the rules)."""
    meta = meta or {}
    if len(shards) == 1:
        return dict(shards[0])
    parts = meta.get("tp_partitions")
    if parts:
        from ..checkpoint.reshape import reshape_tp_states
        return reshape_tp_states([{"module": s, "tp_partitions": parts} for s in shards], 1)[0]["module"]
    out = {}
    n = len(shards)
    for k in shards[0]:
        ts = [s[k] for s in shards]
        if not torch.is_tensor(ts[0]) or ts[0].dim() == 0:
            out[k] = ts[0]
            continue
        want = tuple(full_shapes[k]) if full_shapes is not None and k in full_shapes else None
        same = all(t.shape == ts[0].shape for t in ts)
        if want is None or tuple(ts[0].shape) == want:
            if want is None and same and not all(torch.equal(t, ts[0]) for t in ts[1:]):
                raise ValueError(f"cannot merge {k}: {n} differing shards and no target shape / tp_partitions")
            out[k] = ts[0]
            continue
        dims = [d for d in range(len(want)) if sum(t.shape[d] for t in ts) == want[d]
                and all(t.shape[:d] + t.shape[d + 1:] == ts[0].shape[:d] + ts[0].shape[d + 1:] for t in ts)]
        if not dims or len(want) != ts[0].dim():
            raise ValueError(f"cannot merge {k}: shard shapes {[tuple(t.shape) for t in ts]} vs model {want}")
        out[k] = torch.cat(ts, dim=dims[0])
    return out


def load_state_dict_source(model, source, strict=True):
    """Load ``source`` (see ``read_shards``) into the UNSHARDED ``model``; returns the list of keys
    loaded. Strict: missing or unexpected keys raise ``KeyError`` naming them (a silently random
    layer is worse than a failed start)."""
    shards, meta = read_shards(source)
    target = model.state_dict()
    full = merge_shards(shards, {k: v.shape for k, v in target.items()}, meta)
    missing = sorted(set(target) - set(full))
    unexpected = sorted(set(full) - set(target))
    if strict and (missing or unexpected):
        raise KeyError(f"checkpoint {source if isinstance(source, str) else 'descriptor'} does not match the model: "
                       f"missing {missing[:20]}{' ...' if len(missing) > 20 else ''} ({len(missing)}), "
                       f"unexpected {unexpected[:20]}{' ...' if len(unexpected) > 20 else ''} ({len(unexpected)})")
    bad = [k for k in full if k in target and tuple(full[k].shape) != tuple(target[k].shape)]
    if bad:
        raise ValueError(f"shape mismatch after MP merge: " + ", ".join(
            f"{k} {tuple(full[k].shape)} vs {tuple(target[k].shape)}" for k in bad[:10]))
    model.load_state_dict({k: v for k, v in full.items() if k in target}, strict=False)
    return sorted(k for k in full if k in target)


class SDLoaderFactory:
    """Reference-named facade (runtime/state_dict_factory.py:21)."""

    @staticmethod
    def get_sd_loader_json(json_file, checkpoint_engine=None):
        if isinstance(json_file, str):
            with open(json_file) as f:
                desc = json.load(f)
            desc.setdefault("base_dir", os.path.dirname(os.path.abspath(json_file)))
        else:
            desc = dict(json_file)
        return _Loader(desc)

    @staticmethod
    def get_sd_loader(ckpt_list, checkpoint_engine=None, sd_type="Megatron", version=None):
        return _Loader({"type": sd_type, "checkpoints": list(ckpt_list), "version": version})


class _Loader:
    def __init__(self, desc):
        self.desc = desc

    def load(self, mp_world_size, mp_rank, model=None, **kw):
        """(path, merged-or-split state dict for this MP rank); with ``model`` given the shards are
        merged to its (unsharded) shapes first."""
        shards, meta = read_shards(self.desc)
        if len(shards) == mp_world_size:
            return self.desc.get("checkpoints", [None])[mp_rank], shards[mp_rank]
        full = merge_shards(shards, {k: v.shape for k, v in model.state_dict().items()} if model is not None else None,
                            meta)
        return None, full
