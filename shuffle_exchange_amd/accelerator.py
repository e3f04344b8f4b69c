"""Platform layer: one concrete MI355X (ROCm/HIP) device object.

The reference routes every device call through ``get_accelerator()`` (a ~60-method multi-vendor
abstraction whose source is missing from the snapshot). This framework targets one
platform, so this module is a thin, direct wrapper over ``torch.cuda`` (HIP on ROCm) plus the
pieces the runtime needs: named stream pools, pinned host buffers, graphs, roctx ranges. The only
other mode is a host-CPU mode used by the gloo plumbing tests (no dispatch tables, no op builders).
"""
import contextlib
import os

import torch


class MI355X:
    """Device facade. ``name`` is 'cuda' (PyTorch's name for HIP devices on ROCm) or 'cpu'."""

    def __init__(self):
        self.gpu = torch.cuda.is_available()
        self._name = "cuda" if self.gpu else "cpu"
        self._streams = {}

    # -- identity ---------------------------------------------------------------------------------
    def device_name(self, index=None):
        if index is None or not self.gpu:
            return self._name
        return f"{self._name}:{index}"

    def current_device_name(self):
        return f"cuda:{torch.cuda.current_device()}" if self.gpu else "cpu"

    def current_device(self):
        return torch.cuda.current_device() if self.gpu else 0

    def device(self, index=None):
        return torch.device(self.device_name(index))

    def device_count(self):
        return torch.cuda.device_count() if self.gpu else 1

    def set_device(self, index):
        if self.gpu:
            torch.cuda.set_device(index)

    def is_available(self):
        return self.gpu

    def communication_backend_name(self):
        # torch.distributed's "nccl" backend IS RCCL on ROCm; collectives ride xGMI.
        return "nccl" if self.gpu else "gloo"

    def arch(self):
        if not self.gpu:
            return "cpu"
        return getattr(torch.cuda.get_device_properties(0), "gcnArchName", "gfx950")

    def on_accelerator(self, t):
        return t.device.type == self._name

    # -- sync / streams / events -------------------------------------------------------------------
    def synchronize(self, device=None):
        if self.gpu:
            torch.cuda.synchronize(device)

    def current_stream(self, device=None):
        return torch.cuda.current_stream(device) if self.gpu else None

    def default_stream(self, device=None):
        return torch.cuda.default_stream(device) if self.gpu else None

    def Stream(self, *args, **kw):
        return torch.cuda.Stream(*args, **kw) if self.gpu else None

    def named_stream(self, name, priority=0):
        """A process-wide stream per role ("comm", "allgather", "reduce", "offload", ...).

        Distinct roles get distinct HIP streams so RCCL collectives and D2H/H2D copies overlap
        compute (the reference uses per-optimizer side streams: stage_1_and_2.py:1243,
        partitioned_param_coordinator.py:501)."""
        if not self.gpu:
            return None
        key = (name, torch.cuda.current_device())
        if key not in self._streams:
            self._streams[key] = torch.cuda.Stream(priority=priority)
        return self._streams[key]

    def stream(self, s):
        if s is None or not self.gpu:
            return contextlib.nullcontext()
        return torch.cuda.stream(s)

    def Event(self, **kw):
        return torch.cuda.Event(**kw) if self.gpu else None

    # -- memory -----------------------------------------------------------------------------------
    def memory_allocated(self, device=None):
        return torch.cuda.memory_allocated(device) if self.gpu else 0

    def max_memory_allocated(self, device=None):
        return torch.cuda.max_memory_allocated(device) if self.gpu else 0

    def memory_reserved(self, device=None):
        return torch.cuda.memory_reserved(device) if self.gpu else 0

    def reset_peak_memory_stats(self, device=None):
        if self.gpu:
            torch.cuda.reset_peak_memory_stats(device)

    def total_memory(self, device=None):
        if not self.gpu:
            return 0
        return torch.cuda.get_device_properties(device or 0).total_memory

    def available_memory(self, device=None):
        if not self.gpu:
            return 0
        free, _ = torch.cuda.mem_get_info(device)
        return free

    def empty_cache(self):
        if self.gpu:
            torch.cuda.empty_cache()

    def pin_memory(self, t, align_bytes=1):
        return t.pin_memory() if self.gpu else t

    def is_pinned(self, t):
        return t.is_pinned() if self.gpu else False

    # -- RNG ----------------------------------------------------------------------------------------
    def manual_seed(self, seed):
        torch.manual_seed(seed)
        if self.gpu:
            torch.cuda.manual_seed(seed)

    def manual_seed_all(self, seed):
        torch.manual_seed(seed)
        if self.gpu:
            torch.cuda.manual_seed_all(seed)

    def get_rng_state(self, device=None):
        return torch.cuda.get_rng_state(device or "cuda") if self.gpu else torch.get_rng_state()

    def set_rng_state(self, state, device=None):
        if self.gpu:
            torch.cuda.set_rng_state(state, device or "cuda")
        else:
            torch.set_rng_state(state)

    # -- graphs (hipGraph) --------------------------------------------------------------------------
    def create_graph(self):
        return torch.cuda.CUDAGraph() if self.gpu else None

    def capture_to_graph(self, graph, pool=None, stream=None):
        return torch.cuda.graph(graph, pool=pool, stream=stream)

    def replay_graph(self, graph):
        graph.replay()

    # -- tracing (roctx via torch's nvtx shim on ROCm) ----------------------------------------------
    def range_push(self, msg):
        if self.gpu and os.environ.get("SXE_ROCTX", "0") == "1":
            torch.cuda.nvtx.range_push(msg)

    def range_pop(self):
        if self.gpu and os.environ.get("SXE_ROCTX", "0") == "1":
            torch.cuda.nvtx.range_pop()

    # -- dtype support -----------------------------------------------------------------------------
    def is_bf16_supported(self):
        return True

    def is_fp16_supported(self):
        return True

    def supported_dtypes(self):
        return [torch.float32, torch.bfloat16, torch.float16]

    def use_host_timers(self):
        return not self.gpu

    def resolves_data_dependency(self):
        return False

    def handles_memory_backpressure(self):
        return False


_ACCEL = None


def get_accelerator():
    global _ACCEL
    if _ACCEL is None:
        _ACCEL = MI355X()
    return _ACCEL
