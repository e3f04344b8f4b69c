"""Save / rebuild a ragged inference engine without the original model (reference
inference/v2/engine_v2.py:251 ``serialize`` -> per-TP-rank flattened parameters + metadata, and
inference/v2/engine_factory.py:32-66 ``build_engine_from_ds_checkpoint``).

Layout of ``save_path`` (one set of files per tensor-parallel rank, so a TP=k engine reloads on k
ranks with no re-sharding or re-quantization):

  ds_model_config.json      engine / model description shared by the ranks (implementation, spec or
                            model config, dtype, tp_size, weight_quant)
  params_rank_{r}.pt        {name: tensor} -- ``torch.save`` of plain tensors only, loaded back with
                            ``weights_only=True``
  metadata_rank_{r}.json    per entry: a plain tensor, or a quantized weight object (an allow-listed
                            class: FP8Weight / FPxWeight / IntWeight / MXWeight / QuantizedExperts) whose
                            tensor fields live in the params file and whose scalar fields are here

Nothing is unpickled on load: the quantized objects are re-created from their fields without
running their quantizers again (bit-identical weights).
"""
import dataclasses
import json
import os

import torch

FORMAT = "sxe-v2-1"


def _qclasses():
    from ...ops.fp_quantizer import FP8Weight, FPxWeight
    from ...ops.moe import IntWeight, QuantizedExperts
    from ...ops.mx import MXWeight
    return {c.__name__: c for c in (FP8Weight, FPxWeight, IntWeight, MXWeight, QuantizedExperts)}


def _jsonable(v):
    if isinstance(v, torch.dtype):
        return {"__dtype__": str(v).replace("torch.", "")}
    if isinstance(v, (tuple, list)):
        return {"__tuple__": [_jsonable(x) for x in v]} if isinstance(v, tuple) else [_jsonable(x) for x in v]
    if isinstance(v, torch.Size):
        return {"__tuple__": list(v)}
    if v is None or isinstance(v, (bool, int, float, str)):
        return v
    if isinstance(v, dict):
        return {k: _jsonable(x) for k, x in v.items()}
    raise TypeError(f"cannot serialise field of type {type(v).__name__}")


def _unjson(v):
    if isinstance(v, dict):
        if "__dtype__" in v:
            return getattr(torch, v["__dtype__"])
        if "__tuple__" in v:
            return tuple(_unjson(x) for x in v["__tuple__"])
        return {k: _unjson(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_unjson(x) for x in v]
    return v


def flatten_entries(named):
    """{name: tensor | quantized object} -> (tensors dict, metadata dict)."""
    qc = _qclasses()
    tensors, meta = {}, {}
    for name, v in named.items():
        if torch.is_tensor(v):
            tensors[name] = v.detach().cpu().contiguous()
            meta[name] = {"kind": "tensor"}
        elif type(v).__name__ in qc:
            fields = {}
            for a, x in vars(v).items():
                if torch.is_tensor(x):
                    tensors[f"{name}::{a}"] = x.detach().cpu().contiguous()
                    fields[a] = "tensor"
                else:
                    fields[a] = {"value": _jsonable(x)}
            meta[name] = {"kind": "qobj", "cls": type(v).__name__, "fields": fields}
        elif v is None:
            continue
        else:
            raise TypeError(f"serialize: {name} is a {type(v).__name__}, not a tensor or a known quantized weight")
    return tensors, meta


def restore_entries(tensors, meta, device):
    qc = _qclasses()
    out = {}
    for name, m in meta.items():
        if m["kind"] == "tensor":
            out[name] = tensors[name].to(device)
            continue
        cls = qc[m["cls"]]  # allow-listed classes only
        obj = cls.__new__(cls)
        for a, f in m["fields"].items():
            obj.__dict__[a] = tensors[f"{name}::{a}"].to(device) if f == "tensor" else _unjson(f["value"])
        out[name] = obj
    return out


# ------------------------------------------------------------------------------------------------
def serialize_engine(engine, save_path):
    """Write ``engine``'s model (this rank's shard) under ``save_path`` (every TP rank calls this)."""
    from .model_implementations import RaggedDecoder, RaggedLlama
    os.makedirs(save_path, exist_ok=True)
    m = engine._model
    cfg = engine._config
    common = {"format": FORMAT, "tp_size": int(getattr(m, "tp", 1)), "dtype": str(m.dtype).replace("torch.", ""),
              "kv_block_size": cfg.kv_block_size, "weight_quant": getattr(m, "weight_quant", None)
              or getattr(m, "_weight_quant", None)}
    rank = int(getattr(m, "tp_rank", 0))
    if isinstance(m, RaggedDecoder):
        named = {k: v for k, v in m.w.items() if k != "layers"}
        for i, L in enumerate(m.w["layers"]):
            named.update({f"layers.{i}.{k}": v for k, v in L.items()})
        desc = dict(common, implementation="RaggedDecoder", spec=_jsonable(dataclasses.asdict(m.spec)),
                    n_layers=len(m.w["layers"]))
        rank_meta = {"nq": m.nq, "nkv": m.nkv}
    elif isinstance(m, RaggedLlama):
        named = dict(m.model.state_dict())
        desc = dict(common, implementation="RaggedLlama", model_class=type(m.model).__name__,
                    model_config=_jsonable(dataclasses.asdict(m.model.cfg)), pins=_jsonable(m._pins))
        rank_meta = {}
    else:
        raise NotImplementedError(f"serialize: no format for {type(m).__name__}")
    tensors, meta = flatten_entries(named)
    torch.save(tensors, os.path.join(save_path, f"params_rank_{rank}.pt"))
    with open(os.path.join(save_path, f"metadata_rank_{rank}.json"), "w") as f:
        json.dump({"format": FORMAT, "tp_rank": rank, "entries": meta, **rank_meta}, f)
    if rank == 0:
        with open(os.path.join(save_path, "ds_model_config.json"), "w") as f:
            json.dump(desc, f, indent=1)
    return save_path


def build_engine_from_ds_checkpoint(path, engine_config=None, debug_level=None):
    """Rebuild an InferenceEngineV2 from ``serialize`` output. Run on as many ranks as it was saved
    with (``tensor_parallel.tp_size`` is taken from the checkpoint)."""
    from ... import comm as dist
    from .engine_v2 import InferenceEngineV2, RaggedInferenceEngineConfig, _tp_group
    from .model_implementations import RaggedDecoder, RaggedLlama
    from .model_implementations.hf_decoder import DecoderSpec, _rope_cache
    with open(os.path.join(path, "ds_model_config.json")) as f:
        desc = json.load(f)
    if desc.get("format") != FORMAT:
        raise ValueError(f"{path}: unknown serialization format {desc.get('format')!r}")
    tp = int(desc["tp_size"])
    cfg = engine_config or RaggedInferenceEngineConfig(kv_block_size=desc.get("kv_block_size", 64))
    cfg.tensor_parallel = {"tp_size": tp}
    group = _tp_group(tp) if tp > 1 else None
    rank = dist.get_rank(group) if tp > 1 else 0
    with open(os.path.join(path, f"metadata_rank_{rank}.json")) as f:
        rmeta = json.load(f)
    tensors = torch.load(os.path.join(path, f"params_rank_{rank}.pt"), map_location="cpu", weights_only=True)
    device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    dtype = getattr(torch, desc["dtype"])
    named = restore_entries(tensors, rmeta["entries"], device)
    if desc["implementation"] == "RaggedDecoder":
        sd = _unjson(desc["spec"])
        spec = DecoderSpec(**{k: (tuple(v) if isinstance(v, list) else v) for k, v in sd.items()})
        w = {"layers": [dict() for _ in range(int(desc["n_layers"]))]}
        for k, v in named.items():
            if k.startswith("layers."):
                _, i, key = k.split(".", 2)
                w["layers"][int(i)][key] = v
            else:
                w[k] = v
        m = RaggedDecoder.__new__(RaggedDecoder)
        m.spec, m.tp, m.tp_group, m.tp_rank = spec, tp, group, rank
        m.nq, m.nkv = int(rmeta["nq"]), int(rmeta["nkv"])
        m.w, m.weight_quant = w, desc.get("weight_quant")
        m.num_layers, m.head_dim, m.vocab_size = spec.n_layers, spec.head_dim, spec.vocab_size
        m._dtype, m._device = dtype, device
        m.rope = _rope_cache(spec, device) if spec.rotary_dim else None
        m.scale = spec.head_dim ** -0.5
        m.model = m
    elif desc["implementation"] == "RaggedLlama":
        from ...models.llama import LlamaConfig, LlamaForCausalLM
        from ...models.mixtral import MixtralConfig, MixtralForCausalLM
        classes = {"LlamaForCausalLM": (LlamaForCausalLM, LlamaConfig),
                   "MixtralForCausalLM": (MixtralForCausalLM, MixtralConfig)}
        mcls, ccls = classes[desc["model_class"]]
        mc = _unjson(desc["model_config"])
        model = mcls(ccls(**mc)).to(device=device, dtype=dtype).eval()
        model.load_state_dict(named, strict=True)
        for layer in model.layers:  # served in one process group: routing is local
            moe = getattr(layer, "block_sparse_moe", None)
            if moe is not None:
                moe._groups_ready = True
        m = RaggedLlama(model, weight_quant=desc.get("weight_quant"), tp_group=group, tp_size=tp,
                        pins=_unjson(desc.get("pins")))
    else:
        raise ValueError(f"unknown implementation {desc['implementation']!r}")
    return InferenceEngineV2(m, cfg)
