"""Hybrid engine for RLHF: the same module trains under ZeRO and generates with the ragged,
KV-cached inference path between training steps.

Parity: reference runtime/hybrid_engine.py ``DeepSpeedHybridEngine`` :30 (``generate`` gathering
ZeRO-3 partitions, inference kernels / containers, ``eval`` / ``train`` switching,
``release_inference_cache``, LoRA fuse / unfuse :132-146, inference tensor parallelism
``inference_tp_size``, timing of generate vs train :168-272). Design here: no separate inference copy
of the weights -- ZeRO-3 units are gathered once into their flat buffers for the whole generation
(one all-gather per unit instead of one per token), the ragged engine reads the training modules'
parameters directly, and the units are released afterwards. The KV cache is allocated once and
kept unless ``release_inference_cache`` is set.
"""
import time

import torch

from .engine import SXEEngine


class SXEHybridEngine(SXEEngine):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._he_cfg = self._config.model.hybrid_engine
        self._ragged = None
        self._gen_time = 0.0
        self._train_time = 0.0
        self._t_last = time.perf_counter()

    def _inference_engine(self):
        if self._ragged is None:
            from ..inference.v2 import RaggedInferenceEngineConfig, build_engine
            from ..inference.v2.engine_v2 import MemoryConfig, StateManagerConfig
            cfg = RaggedInferenceEngineConfig(state_manager=StateManagerConfig(
                memory_config=MemoryConfig(fraction=self._he_cfg.kv_cache_fraction)),
                tensor_parallel={"tp_size": int(self._he_cfg.inference_tp_size)})
            if not torch.cuda.is_available():
                cfg.num_kv_blocks = 1024
                cfg.kv_block_size = 16
            self._ragged = build_engine(self.module, cfg)
        elif hasattr(self._ragged.model, "refresh_shards"):
            self._ragged.model.refresh_shards()  # weights moved since the last generation
        return self._ragged

    # ------------------------------------------------------------------------------------ LoRA
    def _lora_modules(self):
        return [m for m in self.module.modules() if hasattr(m, "fuse_lora") and hasattr(m, "unfuse_lora")]

    def fuse_lora_weight(self):
        from ..ops.linear import invalidate_transposed_weights
        for m in self._lora_modules():
            m.fuse_lora()
        invalidate_transposed_weights()  # the base weights changed in place

    def unfuse_lora_weight(self):
        from ..ops.linear import invalidate_transposed_weights
        for m in self._lora_modules():
            m.unfuse_lora()
        invalidate_transposed_weights()

    @torch.no_grad()
    def generate(self, input_ids, max_new_tokens=None, do_sample=False, temperature=1.0, top_k=0, eos_token_id=None,
                 seed=None, **kw):
        t0 = time.perf_counter()
        self._train_time += t0 - self._t_last
        was_training = self.module.training
        self.module.eval()
        z3 = self.zero_optimization_stage() == 3
        if z3:
            self.optimizer.gather_all()
        self.fuse_lora_weight()
        try:
            eng = self._inference_engine()
            prompts = [list(map(int, r)) for r in (input_ids.tolist() if torch.is_tensor(input_ids) else input_ids)]
            n = max_new_tokens or self._he_cfg.max_out_tokens
            outs = eng.generate(prompts, max_new_tokens=n, temperature=temperature if do_sample else 0.0,
                                top_k=top_k, eos_token_id=eos_token_id, seed=seed)
        finally:
            self.unfuse_lora_weight()
            if z3:
                self.optimizer.release_all()
            if self._he_cfg.release_inference_cache:
                self._ragged = None
                if torch.cuda.is_available():
                    torch.cuda.empty_cache()
            self.module.train(was_training)
        width = max(len(p) + len(o) for p, o in zip(prompts, outs))
        pad = eos_token_id if eos_token_id is not None else 0
        res = torch.full((len(prompts), width), pad, dtype=torch.long)
        for i, (p, o) in enumerate(zip(prompts, outs)):
            res[i, :len(p) + len(o)] = torch.tensor(p + o)
        self._t_last = time.perf_counter()
        self._gen_time += self._t_last - t0
        self._gen_tokens = getattr(self, "_gen_tokens", 0) + sum(len(o) for o in outs)
        self._gen_calls = getattr(self, "_gen_calls", 0) + 1
        return res.to(self.device)

    def timing(self):
        return {"generate_s": self._gen_time, "train_s": self._train_time,
                "generated_tokens": getattr(self, "_gen_tokens", 0), "generate_calls": getattr(self, "_gen_calls", 0),
                "generate_tokens_per_s": getattr(self, "_gen_tokens", 0) / max(self._gen_time, 1e-9)}

    def step(self, *args, **kwargs):
        out = super().step(*args, **kwargs)
        spp = self._config.steps_per_print
        if spp and self.global_steps % spp == 0 and getattr(self, "_gen_calls", 0):
            from ..utils.logging import log_dist
            t = self.timing()
            log_dist(f"HybridEngine: step={self.global_steps} generate {t['generate_s']:.2f}s "
                     f"({t['generate_tokens_per_s']:.1f} tok/s over {t['generate_calls']} calls), "
                     f"train {t['train_s']:.2f}s", ranks=[0])
        return out
