"""Hybrid engine for RLHF: the same module trains under ZeRO and generates with the ragged,
KV-cached inference path between training steps.

Parity: reference runtime/hybrid_engine.py ``DeepSpeedHybridEngine`` :30 (``generate`` gathering
ZeRO-3 partitions, inference kernels / containers, ``eval`` / ``train`` switching,
``release_inference_cache``, timing of generate vs train). Design here: no separate inference copy
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
                memory_config=MemoryConfig(fraction=self._he_cfg.kv_cache_fraction)))
            if not torch.cuda.is_available():
                cfg.num_kv_blocks = 1024
                cfg.kv_block_size = 16
            self._ragged = build_engine(self.module, cfg)
        return self._ragged

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
        try:
            eng = self._inference_engine()
            prompts = [list(map(int, r)) for r in (input_ids.tolist() if torch.is_tensor(input_ids) else input_ids)]
            n = max_new_tokens or self._he_cfg.max_out_tokens
            outs = eng.generate(prompts, max_new_tokens=n, temperature=temperature if do_sample else 0.0,
                                top_k=top_k, eos_token_id=eos_token_id, seed=seed)
        finally:
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
        return res.to(self.device)

    def timing(self):
        return {"generate_s": self._gen_time, "train_s": self._train_time}
