"""``init_inference`` engine (v1 API): dtype/device placement, AutoTP sharding, HIP-graph replay of
fixed-shape forwards, and KV-cached ``generate`` through the ragged v2 engine.

Parity: reference inference/engine.py -- ``InferenceEngine`` :40 (``_create_model_parallel_group``
:247, ``_apply_injection_policy`` :378 / AutoTP, ``_create_cuda_graph`` :494, ``forward`` :554,
``_generate``), config inference/config.py ``DeepSpeedInferenceConfig``.
The framework's own models always run the gfx950 kernels. ``replace_with_kernel_inject`` (default
False, as in the reference) swaps Hugging Face layers that have an injection policy for fused gfx950
layers (module_inject/replace_module.py); under ``tp_size > 1`` the fused layers are sliced per rank
(heads of the packed QKV, MLP columns; row-parallel outputs all-reduce), and with post-init weight
quantization their GEMM weights are stored int8 / int4. ``checkpoint`` takes a file, a JSON
descriptor or an ``mp_rank_*`` directory, merged / split to the running TP degree
(runtime/state_dict_factory.py) and loaded strictly. ``generate`` uses the ragged KV-cached engine
whenever the architecture has a v2 implementation (TP 1), independent of injection.
"""
from dataclasses import dataclass, field
from typing import Optional

import torch

from .. import comm as dist
from ..utils.logging import log_dist

_DT = {"fp32": torch.float32, "float32": torch.float32, "fp16": torch.float16, "float16": torch.float16,
       "half": torch.float16, "bf16": torch.bfloat16, "bfloat16": torch.bfloat16}


@dataclass
class InferenceConfig:
    dtype: object = torch.bfloat16
    tensor_parallel: dict = field(default_factory=lambda: {"tp_size": 1})
    replace_with_kernel_inject: bool = False
    enable_cuda_graph: bool = False
    max_out_tokens: int = 1024
    max_tokens: Optional[int] = None
    checkpoint: Optional[str] = None
    mp_size: Optional[int] = None
    kv_block_size: int = 64
    kv_cache_fraction: float = 0.5
    weight_quantization: Optional[dict] = None  # {"post_init_quant": {name-key: {num_bits, group_size, ...}}}
    load_strict: bool = True  # checkpoint keys must match the model exactly (missing / unexpected raise)

    def __post_init__(self):
        if isinstance(self.dtype, str):
            self.dtype = _DT[self.dtype.lower()]
        if self.mp_size is not None:
            self.tensor_parallel = {"tp_size": self.mp_size}
        if isinstance(self.tensor_parallel, int):
            self.tensor_parallel = {"tp_size": self.tensor_parallel}
        if self.max_tokens is not None:
            self.max_out_tokens = self.max_tokens

    @property
    def tp_size(self):
        return int(self.tensor_parallel.get("tp_size", 1))


class _HFWeights:
    """The config + state dict of a Hugging Face model captured before kernel injection (tensor
    references, no copies), in the shape ``ragged_model_for`` accepts."""

    def __init__(self, model):
        self.config = model.config
        self._sd = {k: v.detach() for k, v in model.state_dict().items()}

    @classmethod
    def of(cls, model):
        cfg = getattr(model, "config", None)
        if cfg is None or not hasattr(cfg, "to_dict") or not hasattr(cfg, "model_type"):
            return None
        from .v2.model_implementations.hf_decoder import spec_from_hf_config
        try:
            spec_from_hf_config(cfg.to_dict())
        except Exception:  # not a ragged-decoder family: generate falls back to the module
            return None
        return cls(model)

    def state_dict(self):
        return self._sd

    def parameters(self):
        return (v for v in self._sd.values() if v.is_floating_point())

    def eval(self):
        return self


class InferenceEngine(torch.nn.Module):
    def __init__(self, model, config: InferenceConfig):
        super().__init__()
        self._config = config
        self.module = model
        dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        tp_group = None
        if config.tp_size > 1:
            dist.init_distributed()
            from ..parallel import groups
            groups.initialize(tensor_parallel_size=config.tp_size)
            tp_group = groups.get_tensor_model_parallel_group()
        if config.checkpoint:
            # one file, a JSON descriptor or an mp_rank_* checkpoint directory, merged to the whole model
            # (runtime/state_dict_factory.py) BEFORE any sharding: the TP split below cuts it to this
            # job's degree whatever degree it was saved at; strict unless load_strict=False
            from ..runtime.state_dict_factory import load_state_dict_source
            load_state_dict_source(model, config.checkpoint, strict=config.load_strict)
        self.injected_layers = 0
        self.injection_skipped = None
        self.tp_sharded_layers = 0
        quant = (config.weight_quantization or {}).get("post_init_quant") if config.weight_quantization else None
        if config.replace_with_kernel_inject:
            model.to(device=dev, dtype=config.dtype).eval()
            # Hugging Face layers with an injection policy -> fused gfx950 layers (replace_module.py).
            # The fused layers re-pack their weights, so the KV-cached ragged decoder (built on the
            # first generate) reads the HF tensors as they were before injection.
            self._ragged_src = _HFWeights.of(model) if config.tp_size == 1 and not quant else None
            from ..module_inject.replace_module import (replace_transformer_layer, shard_fused_layers,
                                                        quantize_fused_layer, _Fused)
            from ..module_inject.diffusers import generic_injection
            self.injected_layers = replace_transformer_layer(model)
            # diffusers-style attention (UNet / VAE / transformer blocks; reference
            # generic_injection): fused packed-projection attention modules
            self.injected_layers += generic_injection(model)
            if config.tp_size > 1:
                # reference replace_module.py:207-231: the injected layers' q|k|v heads and MLP columns
                # are sliced per rank, attention-out / MLP-out all-reduce over the TP group
                self.tp_sharded_layers = shard_fused_layers(model, dist.get_rank(tp_group), config.tp_size, tp_group)
                if self.tp_sharded_layers == 0:  # nothing injectable: AutoTP shards the model's linears
                    from ..module_inject.auto_tp import tp_model_init
                    tp_model_init(model, config.tp_size, tp_group=tp_group)
            if quant:
                for name, m in model.named_modules():
                    if isinstance(m, _Fused):
                        names = [name] + [f"{name}.{n}" for n, _ in m.orig.named_modules()] if m.orig is not None \
                            else [name]
                        key = next((k for k in quant if any(k in n for n in names)), None)
                        if key is not None:
                            quantize_fused_layer(m, quant[key])
                from .quantization import _init_group_wise_weight_quantization
                _init_group_wise_weight_quantization(model, {"weight_quantization": config.weight_quantization})
        else:
            if config.tp_size > 1:
                from ..module_inject.auto_tp import tp_model_init
                tp_model_init(model, config.tp_size, tp_group=tp_group)
            model.to(device=dev, dtype=config.dtype).eval()
            if config.weight_quantization:
                from .quantization import _init_group_wise_weight_quantization
                _init_group_wise_weight_quantization(model, {"weight_quantization": config.weight_quantization})
        self.device = dev
        self._graphs = {}
        self._ragged = None
        self._ragged_src = getattr(self, "_ragged_src", None)
        log_dist(f"InferenceEngine: dtype={config.dtype}, tp={config.tp_size}, hip_graph={config.enable_cuda_graph}",
                 ranks=[0])

    # --------------------------------------------------------------------------------- forward
    def _graph_forward(self, *args):
        key = tuple((a.shape, a.dtype) if torch.is_tensor(a) else a for a in args)
        g = self._graphs.get(key)
        if g is None:
            static_in = [a.clone() if torch.is_tensor(a) else a for a in args]
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s), torch.no_grad():
                for _ in range(2):  # warm up allocator / lazy inits outside the capture
                    self.module(*static_in)
            torch.cuda.current_stream().wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph), torch.no_grad():
                static_out = self.module(*static_in)
            g = (graph, static_in, static_out)
            self._graphs[key] = g
        graph, static_in, static_out = g
        for dst, src in zip(static_in, args):
            if torch.is_tensor(src):
                dst.copy_(src)
        graph.replay()
        return static_out

    @torch.no_grad()
    def forward(self, *args, **kwargs):
        if self._config.enable_cuda_graph and self.device.type == "cuda" and not kwargs:
            return self._graph_forward(*args)
        return self.module(*args, **kwargs)

    # -------------------------------------------------------------------------------- generate
    def _ragged_engine(self):
        if self._ragged is None:
            from .v2 import RaggedInferenceEngineConfig, build_engine
            from .v2.engine_v2 import MemoryConfig, StateManagerConfig
            cfg = RaggedInferenceEngineConfig(
                kv_block_size=self._config.kv_block_size,
                state_manager=StateManagerConfig(memory_config=MemoryConfig(fraction=self._config.kv_cache_fraction)))
            if self.device.type != "cuda":
                cfg.num_kv_blocks = 1024
            try:
                self._ragged = build_engine(self._ragged_src or self.module, cfg)
            except (KeyError, ValueError) as e:  # an architecture the ragged decoder does not describe
                raise NotImplementedError(f"no ragged KV-cache implementation: {e}") from e
            self._ragged_src = None  # the ragged decoder holds its own packed copy now
        return self._ragged

    @torch.no_grad()
    def generate(self, input_ids, max_new_tokens=None, do_sample=False, temperature=1.0, top_k=0, eos_token_id=None,
                 seed=None, **kw):
        """input_ids: [B, S] (or list of lists). Returns [B, S + new] (prompt + generated)."""
        max_new = max_new_tokens or kw.get("max_length", self._config.max_out_tokens)
        prompts = [list(map(int, r)) for r in (input_ids.tolist() if torch.is_tensor(input_ids) else input_ids)]
        try:
            # AutoTP-sharded models decode through their own (all-reducing) forward
            eng = self._ragged_engine() if self._config.tp_size == 1 else None
        except NotImplementedError:
            eng = None
        if eng is not None:
            outs = eng.generate(prompts, max_new_tokens=max_new, temperature=temperature if do_sample else 0.0,
                                top_k=top_k, eos_token_id=eos_token_id, seed=seed)
        else:  # no KV-cache implementation for this architecture: full recompute per token
            outs = []
            for p in prompts:
                ids = torch.tensor([p], device=self.device)
                gen = []
                for _ in range(max_new):
                    logits = self.module(ids)
                    logits = getattr(logits, "logits", logits)  # Hugging Face ModelOutput
                    logits = logits[0] if isinstance(logits, tuple) else logits
                    nxt = int(logits[0, -1].argmax())
                    gen.append(nxt)
                    ids = torch.cat([ids, torch.tensor([[nxt]], device=self.device)], dim=1)
                    if eos_token_id is not None and nxt == eos_token_id:
                        break
                outs.append(gen)
        width = max(len(p) + len(o) for p, o in zip(prompts, outs))
        pad = eos_token_id if eos_token_id is not None else 0
        res = torch.full((len(prompts), width), pad, dtype=torch.long)
        for i, (p, o) in enumerate(zip(prompts, outs)):
            seq = p + o
            res[i, :len(seq)] = torch.tensor(seq)
        return res.to(self.device)
