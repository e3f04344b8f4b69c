"""Communication facade over torch.distributed (RCCL over xGMI on MI355X; gloo for CPU tests).

Parity: reference deepspeed/comm/comm.py (ops :177-640, ``init_distributed`` :643-709, comms
logger via ``timed_op`` :102-135) and deepspeed/comm/torch.py (``TorchBackend`` :96-421, the
``DS_COMM_*_OFF`` debug toggles :16-88). Differences that matter on MI355X:

* ``isend``/``irecv`` are truly asynchronous (the reference facade calls the blocking send/recv,
  comm/comm.py:380-389 -- a known quirk).
* a **group cache** keyed by the member-rank tuple: RCCL communicator creation costs ~100 ms,
  so the Shuffle-exchange reshuffle (reference stage_1_and_2.py:698-711 destroys and recreates
  every communicator) reuses groups it has seen before.
* a **collective fingerprint**: every collective folds (op, group, numel, dtype) into a per-rank
  running hash; ``verify_fingerprints()`` all-gathers the hashes and raises on divergence. This is
  the race/ordering detector SURVEY §5.2 asks for (it catches e.g. ranks whose shuffle RNG
  diverged, which deadlocks or silently mis-averages in the reference).
* a comms logger reporting per-op latency, algbw and busbw (busbw uses the ring factors of each
  collective, so it is directly comparable to the per-link xGMI bandwidth), and always-on per-op
  byte counters (``get_comm_volume``, no device sync) that bench.py reports per step.
* a test-only **deferred-completion mode** (``set_deferred_completion`` / SXE_COMM_DEFER=1): every
  collective's output reads as NaN until the consumer has synchronised with it -- for device
  tensors, the true result lands on the issuing stream only after a spin delay, so a consumer on
  another stream that skipped its ``wait_event``/``wait_stream`` reads NaN; for async host ops the
  result appears at ``Work.wait()``. The gloo parity suites run under it to prove every consumer of
  an overlapped collective synchronises before RCCL ever runs the code (RCCL completes
  asynchronously on its own stream; gloo and world-size-1 shortcuts complete immediately).
"""
import datetime
import hashlib
import os
import time
from collections import defaultdict

import torch
import torch.distributed as tdist

from ..utils.logging import logger, log_dist

ReduceOp = tdist.ReduceOp

_COMM_OFF = {k: os.environ.get(f"SXE_COMM_{k}_OFF", os.environ.get(f"DS_COMM_{k}_OFF", "0")) == "1"
             for k in ("ALL_GATHER", "REDUCE_SCATTER", "BROADCAST", "ALL_REDUCE", "REDUCE", "ALL_TO_ALL")}


class _State:
    initialized = False
    backend = None
    group_cache = {}
    fingerprint = hashlib.sha1()
    fp_count = 0
    fingerprint_enabled = os.environ.get("SXE_COMM_FINGERPRINT", "0") == "1"
    logger_enabled = False
    logger_verbose = False
    logger_prof_all = True
    logger_prof_ops = []
    comms = defaultdict(lambda: defaultdict(list))  # op -> msg_size -> [latency_ms...]
    op_counts = defaultdict(int)  # log_name -> collectives issued (always counted, no sync)
    volume = defaultdict(lambda: [0, 0])  # op -> [calls, payload bytes] (always counted, no sync)
    group_init = []  # (cache key, ms) per communicator created by new_group
    init_ms = None  # init_process_group wall time
    defer = os.environ.get("SXE_COMM_DEFER", "0") == "1"
    defer_cycles = int(os.environ.get("SXE_COMM_DEFER_CYCLES", 2_000_000))


# ------------------------------------------------------------------------------------------------
# init / identity
def init_distributed(dist_backend=None, auto_mpi_discovery=True, distributed_port=29500, verbose=True,
                     timeout=None, init_method=None, dist_init_required=None, config=None, rank=-1,
                     world_size=-1):
    """Initialise the default process group from the torchrun/launcher env (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR, MASTER_PORT); falls back to OpenMPI env discovery; a single process
    without env becomes a world of one (rendezvous on 127.0.0.1)."""
    from ..accelerator import get_accelerator
    if config is not None:
        configure(config)
    if tdist.is_initialized():
        _State.initialized = True
        _State.backend = tdist.get_backend()
        return
    if dist_init_required is False:
        return
    env = os.environ
    if "RANK" not in env and auto_mpi_discovery and "OMPI_COMM_WORLD_RANK" in env:
        env["RANK"] = env["OMPI_COMM_WORLD_RANK"]
        env["WORLD_SIZE"] = env["OMPI_COMM_WORLD_SIZE"]
        env["LOCAL_RANK"] = env.get("OMPI_COMM_WORLD_LOCAL_RANK", "0")
    if rank >= 0:
        env["RANK"] = str(rank)
    if world_size > 0:
        env["WORLD_SIZE"] = str(world_size)
    env.setdefault("RANK", "0")
    env.setdefault("WORLD_SIZE", "1")
    env.setdefault("LOCAL_RANK", "0")
    # a world of one with no rendezvous given (a single-GPU job, a test process) needs no TCP store:
    # an in-process HashStore means two such processes on one machine never meet at a shared
    # default port (a collision there hangs both in the store handshake)
    solo = (int(env["WORLD_SIZE"]) == 1 and init_method is None and "MASTER_PORT" not in env)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    if not solo:
        env.setdefault("MASTER_PORT", str(distributed_port))
    # SXE_DIST_BACKEND=gloo: multi-rank rehearsals on a single GPU (RCCL needs one GPU per rank)
    backend = dist_backend or env.get("SXE_DIST_BACKEND") or get_accelerator().communication_backend_name()
    if timeout is None:
        timeout = datetime.timedelta(minutes=int(env.get("SXE_TIMEOUT_MIN", env.get("DEEPSPEED_TIMEOUT", "30"))))
    kw = {}
    if backend == "nccl":
        local_rank = int(env["LOCAL_RANK"])
        torch.cuda.set_device(local_rank)
        # binding the device lets RCCL split sub-communicators from the world comm (cheap new_group)
        kw["device_id"] = torch.device("cuda", local_rank)
    if solo:
        kw["store"] = tdist.HashStore()
    else:
        kw["init_method"] = init_method
    t0 = time.perf_counter()
    tdist.init_process_group(backend=backend, timeout=timeout, rank=int(env["RANK"]),
                             world_size=int(env["WORLD_SIZE"]), **kw)
    _State.init_ms = (time.perf_counter() - t0) * 1000.0
    _State.initialized = True
    _State.backend = backend
    if verbose:
        log_dist(f"initialized {backend} world_size={tdist.get_world_size()}", ranks=[0])


def is_initialized():
    return tdist.is_available() and tdist.is_initialized()


def get_rank(group=None):
    return tdist.get_rank(group) if is_initialized() else 0


def get_world_size(group=None):
    return tdist.get_world_size(group) if is_initialized() else 1


def get_local_rank():
    return int(os.environ.get("LOCAL_RANK", 0))


def get_global_rank(group, group_rank):
    return tdist.get_global_rank(group, group_rank) if group is not None else group_rank


def get_backend(group=None):
    return tdist.get_backend(group) if is_initialized() else None


def get_world_group():
    return tdist.group.WORLD


def destroy_process_group(group=None):
    if group is None:
        _State.group_cache.clear()
    else:
        for k, v in list(_State.group_cache.items()):
            if v is group:
                del _State.group_cache[k]
    tdist.destroy_process_group(group)


def new_group(ranks, cache=True, tag=None):
    """Collective over the world (every rank must call with the same `ranks`, in the same order).
    Cached per rank tuple so repeated topologies do not re-create RCCL communicators. ``tag`` names
    a second, independent communicator over the same ranks (e.g. ZeRO-3's gradient reduce-scatter
    next to its parameter all-gathers: ProcessGroupNCCL runs every collective of one communicator
    on one internal stream, so two streams of work on one group serialise)."""
    ranks_key = tuple(sorted(int(r) for r in ranks))
    key = (tag,) + ranks_key if tag is not None else ranks_key
    if cache and key in _State.group_cache:
        return _State.group_cache[key]
    if not is_initialized():
        return None
    t0 = time.perf_counter()
    g = tdist.new_group(list(ranks_key))
    _State.group_init.append((key, (time.perf_counter() - t0) * 1000.0))
    if cache:
        _State.group_cache[key] = g
    return g


def group_ranks(group):
    if group is None or group is tdist.group.WORLD:
        return list(range(get_world_size()))
    return tdist.get_process_group_ranks(group)


# ------------------------------------------------------------------------------------------------
# logging / fingerprint
def configure(config=None, enabled=None, prof_all=None, prof_ops=None, verbose=None):
    if config is not None and getattr(config, "comms_logger", None) is not None:
        cl = config.comms_logger
        _State.logger_enabled = cl.enabled
        _State.logger_prof_all = cl.prof_all
        _State.logger_prof_ops = list(cl.prof_ops)
        _State.logger_verbose = cl.verbose
    if enabled is not None:
        _State.logger_enabled = enabled
    if prof_all is not None:
        _State.logger_prof_all = prof_all
    if prof_ops is not None:
        _State.logger_prof_ops = list(prof_ops)
    if verbose is not None:
        _State.logger_verbose = verbose


def enable_fingerprint(on=True):
    _State.fingerprint_enabled = on


def _fp(op, group, t):
    if not _State.fingerprint_enabled:
        return
    ranks = tuple(group_ranks(group)) if is_initialized() else (0,)
    numel = t.numel() if isinstance(t, torch.Tensor) else sum(x.numel() for x in t)
    dtype = t.dtype if isinstance(t, torch.Tensor) else t[0].dtype
    _State.fingerprint.update(f"{op}|{ranks}|{numel}|{dtype};".encode())
    _State.fp_count += 1


def fingerprint_digest():
    return _State.fingerprint.hexdigest(), _State.fp_count


def verify_fingerprints(group=None):
    """All-gather every rank's collective fingerprint; raise if any rank issued a different
    sequence of collectives (op/group/shape/dtype) since the last reset."""
    if not is_initialized() or get_world_size(group) == 1:
        return True
    digest, count = fingerprint_digest()
    objs = [None] * get_world_size(group)
    tdist.all_gather_object(objs, (digest, count), group=group)
    if len(set(objs)) != 1:
        raise RuntimeError(f"sxe: collective fingerprint mismatch across ranks: {objs}")
    return True


def reset_fingerprint():
    _State.fingerprint = hashlib.sha1()
    _State.fp_count = 0


def _bus_factor(op, n):
    if n <= 1:
        return 1.0
    if op in ("all_reduce", "all_reduce_coalesced"):
        return 2.0 * (n - 1) / n
    if op in ("all_gather_into_tensor", "all_gather", "reduce_scatter_tensor", "reduce_scatter", "all_to_all_single"):
        return (n - 1) / n
    return 1.0


def _payload(op, tensor, group):
    size = (tensor.numel() * tensor.element_size()) if isinstance(tensor, torch.Tensor) else \
        sum(x.numel() * x.element_size() for x in tensor)
    if op in ("all_gather_into_tensor", "all_gather"):
        size *= get_world_size(group)
    return size


def get_comm_volume():
    """{op: (calls, payload bytes)} since the last ``reset_comms_stats()``. Payload as in
    rccl-tests: the gathered output for all-gathers, the input for reduce-scatter / all-reduce /
    all-to-all / broadcast, the message for point-to-point."""
    return {op: (v[0], v[1]) for op, v in _State.volume.items()}


def set_deferred_completion(on=True, cycles=None):
    _State.defer = bool(on)
    if cycles is not None:
        _State.defer_cycles = int(cycles)


class _DeferredWork:
    """Async handle whose result becomes visible at ``wait()`` (deferred-completion mode)."""

    def __init__(self, work, finish):
        self._work, self._finish = work, finish

    def wait(self, timeout=None):
        if self._work is not None:
            self._work.wait()
            self._work = None
        if self._finish is not None:
            self._finish()
            self._finish = None
        return True

    def is_completed(self):
        return self._finish is None


def _deferred(fn, outs, async_op):
    """Run ``fn`` (synchronously), then hide the result of every tensor in ``outs`` until the
    consumer has synchronised: device tensors get NaN now and the result after a spin delay on the
    issuing stream; host tensors of async ops get NaN until ``wait()``."""
    r = fn()
    if r is not None and hasattr(r, "wait"):
        r.wait()
    outs = [t for t in outs if isinstance(t, torch.Tensor) and t.is_floating_point() and t.numel()]
    if not outs:
        return _DeferredWork(None, None) if async_op else None
    stash = [t.clone() for t in outs]
    for t in outs:
        t.fill_(float("nan"))
    if outs[0].is_cuda:
        stream = torch.cuda.current_stream(outs[0].device)
        torch.cuda._sleep(_State.defer_cycles)
        for t, s in zip(outs, stash):
            t.copy_(s)
        if not async_op:
            return None
        ev = torch.cuda.Event()
        ev.record(stream)
        return _DeferredWork(None, lambda: torch.cuda.current_stream(outs[0].device).wait_event(ev))
    if not async_op:  # a blocking host collective has completed when it returns
        for t, s in zip(outs, stash):
            t.copy_(s)
        return None

    def finish():
        for t, s in zip(outs, stash):
            t.copy_(s)
    return _DeferredWork(None, finish)


def _timed(op, fn, tensor, group, async_op, outs=None):
    _fp(op, group, tensor)
    if op != "all_reduce":  # all_reduce counts under its caller's log_name
        _State.op_counts[op] += 1
    v = _State.volume[op]
    v[0] += 1
    v[1] += _payload(op, tensor, group)
    if _State.defer and outs is not None:
        return _deferred(fn, outs, async_op)
    if not _State.logger_enabled or async_op or (not _State.logger_prof_all and op not in _State.logger_prof_ops):
        return fn()
    from ..accelerator import get_accelerator
    acc = get_accelerator()
    acc.synchronize()
    t0 = time.perf_counter()
    r = fn()
    acc.synchronize()
    ms = (time.perf_counter() - t0) * 1000.0
    size = _payload(op, tensor, group)
    _State.comms[op][size].append(ms)
    if _State.logger_verbose:
        n = get_world_size(group)
        algbw = size / (ms / 1000.0) / 1e9 if ms > 0 else 0.0
        log_dist(f"comm op: {op} | time (ms): {ms:.3f} | msg size: {size} | algbw (GB/s): {algbw:.2f} | "
                 f"busbw (GB/s): {algbw * _bus_factor(op, n):.2f}", ranks=[0])
    return r


def log_summary(show_straggler=False):
    """Print the per-op table: count, total/avg latency, algbw/busbw (reference
    utils/comms_logging.py:67)."""
    n = get_world_size()
    lines = [f"{'op':<24}{'msg size':>14}{'count':>8}{'total ms':>12}{'avg ms':>10}{'algbw GB/s':>12}{'busbw GB/s':>12}"]
    for op, d in sorted(_State.comms.items()):
        for size, lat in sorted(d.items()):
            avg = sum(lat) / len(lat)
            algbw = size / (avg / 1000.0) / 1e9 if avg > 0 else 0.0
            lines.append(f"{op:<24}{size:>14}{len(lat):>8}{sum(lat):>12.3f}{avg:>10.3f}{algbw:>12.2f}"
                         f"{algbw * _bus_factor(op, n):>12.2f}")
    log_dist("\n" + "\n".join(lines), ranks=[0])
    return lines


def get_comms_stats():
    return {op: {s: list(v) for s, v in d.items()} for op, d in _State.comms.items()}


def reset_comms_stats():
    _State.comms.clear()
    _State.op_counts.clear()
    _State.volume.clear()


def get_init_times():
    """Wall time of ``init_process_group`` and of every ``new_group`` (RCCL comm split / init) so far:
    ``{"init_process_group_ms": ms, "groups": [(ranks, ms), ...]}``."""
    return {"init_process_group_ms": _State.init_ms,
            "groups": [(list(k), round(ms, 3)) for k, ms in _State.group_init]}


def get_op_counts():
    """Collectives issued per ``log_name`` since the last ``reset_comms_stats()``."""
    return dict(_State.op_counts)


# ------------------------------------------------------------------------------------------------
# collectives
def _skip(kind):
    return _COMM_OFF.get(kind, False)


def all_reduce(tensor, op=ReduceOp.SUM, group=None, async_op=False, prof=False, log_name="all_reduce"):
    if _skip("ALL_REDUCE") or get_world_size(group) == 1:
        return None
    _State.op_counts[log_name] += 1
    return _timed("all_reduce", lambda: tdist.all_reduce(tensor, op=op, group=group, async_op=async_op), tensor,
                  group, async_op, outs=[tensor])


def inference_all_reduce(tensor, op=ReduceOp.SUM, group=None):
    return all_reduce(tensor, op, group)


def all_reduce_coalesced(tensors, op=ReduceOp.SUM, group=None, async_op=False):
    if _skip("ALL_REDUCE") or get_world_size(group) == 1:
        return None
    return _timed("all_reduce_coalesced",
                  lambda: tdist.all_reduce_coalesced(tensors, op=op, group=group, async_op=async_op), tensors, group,
                  async_op, outs=list(tensors))


def reduce(tensor, dst, op=ReduceOp.SUM, group=None, async_op=False):
    if _skip("REDUCE") or get_world_size(group) == 1:
        return None
    return _timed("reduce", lambda: tdist.reduce(tensor, dst, op=op, group=group, async_op=async_op), tensor, group,
                  async_op, outs=[tensor])


def reduce_scatter_tensor(output, input, op=ReduceOp.SUM, group=None, async_op=False):
    if _skip("REDUCE_SCATTER"):
        return None
    if get_world_size(group) == 1:
        if output.data_ptr() != input.data_ptr():
            output.copy_(input.view_as(output))
        return None
    if get_backend(group) == "gloo":
        # gloo lacks reduce_scatter_tensor: all_reduce + slice (plumbing tests only)
        def fn():
            buf = input.clone()
            tdist.all_reduce(buf, op=op, group=group)
            r = get_rank(group)
            output.copy_(buf.view(get_world_size(group), -1)[r].view_as(output))
        return _timed("reduce_scatter_tensor", fn, input, group, False, outs=[output])
    return _timed("reduce_scatter_tensor",
                  lambda: tdist.reduce_scatter_tensor(output, input, op=op, group=group, async_op=async_op), input,
                  group, async_op, outs=[output])


reduce_scatter_fn = reduce_scatter_tensor


def all_gather_into_tensor(output, input, group=None, async_op=False):
    if _skip("ALL_GATHER"):
        return None
    if get_world_size(group) == 1:
        if output.data_ptr() != input.data_ptr():
            output.copy_(input.view_as(output))
        return None
    if get_backend(group) == "gloo":
        def fn():
            parts = list(output.view(get_world_size(group), -1).unbind(0))
            tdist.all_gather(parts, input.reshape(-1), group=group)
        return _timed("all_gather_into_tensor", fn, input, group, False, outs=[output])
    return _timed("all_gather_into_tensor",
                  lambda: tdist.all_gather_into_tensor(output, input, group=group, async_op=async_op), input, group,
                  async_op, outs=[output])


allgather_fn = all_gather_into_tensor


def all_gather(tensor_list, tensor, group=None, async_op=False):
    if _skip("ALL_GATHER"):
        return None
    return _timed("all_gather", lambda: tdist.all_gather(tensor_list, tensor, group=group, async_op=async_op), tensor,
                  group, async_op, outs=list(tensor_list))


def all_gather_object(obj_list, obj, group=None):
    return tdist.all_gather_object(obj_list, obj, group=group)


def broadcast(tensor, src, group=None, async_op=False):
    if _skip("BROADCAST") or get_world_size(group) == 1:
        return None
    return _timed("broadcast", lambda: tdist.broadcast(tensor, src, group=group, async_op=async_op), tensor, group,
                  async_op, outs=[tensor])


def broadcast_object_list(objs, src, group=None):
    if get_world_size(group) == 1:
        return
    tdist.broadcast_object_list(objs, src, group=group)


def all_to_all_single(output, input, output_split_sizes=None, input_split_sizes=None, group=None, async_op=False):
    if _skip("ALL_TO_ALL"):
        return None
    if get_world_size(group) == 1:
        output.copy_(input)
        return None
    return _timed("all_to_all_single",
                  lambda: tdist.all_to_all_single(output, input, output_split_sizes, input_split_sizes, group=group,
                                                  async_op=async_op), input, group, async_op, outs=[output])


def all_to_all(output_tensor_list, input_tensor_list, group=None, async_op=False):
    return tdist.all_to_all(output_tensor_list, input_tensor_list, group=group, async_op=async_op)


def _count_p2p(op, tensor):
    v = _State.volume[op]
    v[0] += 1
    v[1] += tensor.numel() * tensor.element_size()


def send(tensor, dst, group=None, tag=0):
    _fp("send", None, tensor)
    _count_p2p("send", tensor)
    return tdist.send(tensor, dst, group=group, tag=tag)


def recv(tensor, src=None, group=None, tag=0):
    _fp("recv", None, tensor)
    return tdist.recv(tensor, src, group=group, tag=tag)


def isend(tensor, dst, group=None, tag=0):
    _fp("isend", None, tensor)
    _count_p2p("send", tensor)
    return tdist.isend(tensor, dst, group=group, tag=tag)


def irecv(tensor, src=None, group=None, tag=0):
    _fp("irecv", None, tensor)
    if _State.defer and tensor.is_floating_point():
        priv = torch.empty_like(tensor)
        return _DeferredRecv(tdist.irecv(priv, src, group=group, tag=tag), tensor, priv)
    return tdist.irecv(tensor, src, group=group, tag=tag)


class _DeferredRecv(_DeferredWork):
    """irecv under deferred completion: the message lands in a private buffer and the user's
    tensor reads NaN until ``wait()`` copies it over."""

    def __init__(self, work, tensor, priv):
        tensor.fill_(float("nan"))
        super().__init__(work, lambda: tensor.copy_(priv))


def batch_isend_irecv(p2p_op_list):
    ops, wrap = [], []
    for o in p2p_op_list:
        is_recv = o.op in (tdist.irecv, irecv)
        if not is_recv:
            _count_p2p("send", o.tensor)
        if _State.defer and is_recv and o.tensor.is_floating_point():
            priv = torch.empty_like(o.tensor)
            ops.append(tdist.P2POp(tdist.irecv, priv, o.peer, o.group, o.tag))
            wrap.append((o.tensor, priv))
        else:
            ops.append(o)
            wrap.append(None)
    works = tdist.batch_isend_irecv(ops)
    return [w if x is None else _DeferredRecv(w, x[0], x[1]) for w, x in zip(works, wrap)]


P2POp = tdist.P2POp


def barrier(group=None, async_op=False, device_ids=None):
    if not is_initialized():
        return None
    return tdist.barrier(group=group, async_op=async_op)


def monitored_barrier(group=None, timeout=None, wait_all_ranks=False):
    if not is_initialized():
        return None
    if get_backend(group) == "gloo":
        return tdist.monitored_barrier(group=group, timeout=timeout, wait_all_ranks=wait_all_ranks)
    return tdist.barrier(group=group)


def has_reduce_scatter_tensor():
    return True


def has_all_gather_into_tensor():
    return True


# ------------------------------------------------------------------------------------------------
# the rest of the reference facade (deepspeed/comm/comm.py): list-form collectives, capability
# queries, environment discovery and the timing decorator
def is_available():
    return tdist.is_available()


def set_backend(backend_name=None):
    """Select the backend ``init_distributed`` uses when none is passed (reference set_backend)."""
    if backend_name:
        os.environ["SXE_DIST_BACKEND"] = backend_name


def init_deepspeed_backend(ds_backend=None, timeout=None, init_method=None):
    """Reference name for bringing up the communication backend: here always torch.distributed
    (RCCL over xGMI for GPU tensors, gloo for CPU plumbing)."""
    init_distributed(dist_backend=ds_backend, timeout=timeout, init_method=init_method)


def get_all_ranks_from_group(group=None):
    return group_ranks(group)


def has_all_reduce_coalesced():
    return hasattr(tdist, "all_reduce_coalesced")


def has_coalescing_manager():
    return hasattr(tdist, "_coalescing_manager")


def all_gather_coalesced(output_tensors, input_tensors, group=None, async_op=False):
    """Gather several tensors at once: their flat concatenation in ONE all-gather (one RCCL launch
    instead of one per tensor), split back into ``output_tensors[i]`` ([world * numel_i] each)."""
    n = get_world_size(group)
    if n == 1:
        for o, i in zip(output_tensors, input_tensors):
            o.copy_(i.reshape(o.shape))
        return None
    flat = torch.cat([t.reshape(-1) for t in input_tensors])
    out = torch.empty(n * flat.numel(), dtype=flat.dtype, device=flat.device)
    all_gather_into_tensor(out, flat, group=group)
    rows = out.view(n, -1)
    o = 0
    for dst, src in zip(output_tensors, input_tensors):
        k = src.numel()
        dst.view(n, k).copy_(rows[:, o:o + k])
        o += k
    return None


def gather(tensor, gather_list=None, dst=0, group=None, async_op=False):
    if get_world_size(group) == 1:
        if gather_list:
            gather_list[0].copy_(tensor)
        return None
    return _timed("gather", lambda: tdist.gather(tensor, gather_list, dst=dst, group=group, async_op=async_op), tensor,
                  group, async_op)


def scatter(tensor, scatter_list=None, src=0, group=None, async_op=False):
    if get_world_size(group) == 1:
        if scatter_list:
            tensor.copy_(scatter_list[0])
        return None
    return _timed("scatter", lambda: tdist.scatter(tensor, scatter_list, src=src, group=group, async_op=async_op),
                  tensor, group, async_op, outs=[tensor])


def reduce_scatter(output, input_list, op=ReduceOp.SUM, group=None, async_op=False):
    """List form: the inputs are concatenated and reduce-scattered as one tensor (the reference
    calls the backend's list reduce_scatter; one contiguous RCCL call is cheaper on xGMI)."""
    flat = torch.cat([t.reshape(-1) for t in input_list])
    return reduce_scatter_tensor(output.view(-1), flat, op=op, group=group, async_op=async_op)


def timed_op(func):
    """Decorator recording a call's wall time and payload in the comms logger (reference
    comm.py timed_op); the facade's own collectives log through ``_timed`` already."""
    import functools

    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        t = kwargs.get("tensor", args[0] if args and torch.is_tensor(args[0]) else None)
        if t is None or not torch.is_tensor(t):
            return func(*args, **kwargs)
        return _timed(func.__name__, lambda: func(*args, **kwargs), t, kwargs.get("group"), False)
    return wrapper


def mpi_discovery(distributed_port=29500, verbose=True):
    """RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* from an MPI launcher's environment (OpenMPI,
    MPICH / Intel MPI PMI, Slurm), without mpi4py: the launcher env is enough on one node and the
    multinode runners export MASTER_ADDR themselves."""
    env = os.environ
    for rk, ws, lr in (("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK"),
                       ("PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID"), ("SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID")):
        if rk in env:
            env["RANK"], env["WORLD_SIZE"] = env[rk], env.get(ws, "1")
            env["LOCAL_RANK"] = env.get(lr, "0")
            break
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env.setdefault("MASTER_PORT", str(distributed_port))
    if verbose:
        log_dist(f"mpi_discovery: rank {env.get('RANK')} / {env.get('WORLD_SIZE')}", ranks=[0])


def in_aml():
    return "AZUREML_EXPERIMENT_ID" in os.environ


def in_aws_sm():
    return "SM_TRAINING_ENV" in os.environ


def in_dlts():
    return "DLTS_JOB_ID" in os.environ


def patch_aml_env_for_torch_nccl_backend(master_port=6105, verbose=True):
    """AzureML: derive the torch.distributed rendezvous env from its OpenMPI variables."""
    env = os.environ
    env.setdefault("RANK", env.get("OMPI_COMM_WORLD_RANK", "0"))
    env.setdefault("WORLD_SIZE", env.get("OMPI_COMM_WORLD_SIZE", "1"))
    env.setdefault("LOCAL_RANK", env.get("OMPI_COMM_WORLD_LOCAL_RANK", "0"))
    env.setdefault("MASTER_ADDR", env.get("AZ_BATCH_MASTER_NODE", "127.0.0.1:").split(":")[0] or "127.0.0.1")
    env.setdefault("MASTER_PORT", str(master_port))


def patch_aws_sm_env_for_torch_nccl_backend(verbose=True):
    """SageMaker: the same from its OpenMPI variables."""
    env = os.environ
    env.setdefault("RANK", env.get("OMPI_COMM_WORLD_RANK", "0"))
    env.setdefault("WORLD_SIZE", env.get("OMPI_COMM_WORLD_SIZE", "1"))
    env.setdefault("LOCAL_RANK", env.get("OMPI_COMM_WORLD_LOCAL_RANK", "0"))


def initialize_mesh_device(mesh_shape, mesh_dim_names):
    """A torch DeviceMesh over the world (reference initialize_mesh_device); device type from the
    accelerator (cuda on ROCm = the HIP devices)."""
    from torch.distributed.device_mesh import init_device_mesh
    dev = "cuda" if torch.cuda.is_available() and get_backend() == "nccl" else "cpu"
    return init_device_mesh(dev, tuple(mesh_shape), mesh_dim_names=tuple(mesh_dim_names))


def enable_symm_mem_for_group(group_name):
    """Symmetric-memory collectives are a CUDA/NVSHMEM feature; RCCL over xGMI needs no opt-in here
    -- kept for API parity, it only records the request."""
    _State.symm_mem_groups = getattr(_State, "symm_mem_groups", set()) | {group_name}
