"""Per-rank host resources for the host-offload tiers: CPU threads, NUMA placement, memory pre-flight.

One MI355X node runs 8 ranks on one host. The C++ host optimizer (csrc/cpu/cpu_adam.cpp) is DRAM
bound, so what matters per rank is (a) a thread team that is this rank's share of the host, not the
whole host (8 x oversubscription) and not one thread (torchrun exports ``OMP_NUM_THREADS=1`` for
nproc > 1 when the variable is unset), (b) those threads and the fp32 state on the NUMA node the
rank's GPU hangs off, and (c) a clear error before the pinned tier is allocated when the node does
not have the memory -- never an OOM kill half-way through the allocation.

Parity: reference launcher/launch.py:93,230-232 (``OMP_NUM_THREADS = cores per rank`` when binding,
utils/numa.py core lists), runtime/zero/stage_1_and_2.py:1390-1481 (host buffers of the offload path,
which the reference allocates without a check).
"""
import os

from .logging import log_dist


def _local_world():
    for k in ("LOCAL_WORLD_SIZE", "LOCAL_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE"):
        if os.environ.get(k):
            return max(1, int(os.environ[k]))
    return 1


def _local_rank():
    return int(os.environ.get("LOCAL_RANK", 0))


def _parse_cpulist(s):
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _online_cpus():
    try:
        with open("/sys/devices/system/cpu/online") as f:
            return set(_parse_cpulist(f.read()))
    except OSError:
        return set(range(os.cpu_count() or 1))


def gpu_numa_node(device=None):
    """NUMA node of a GPU from its PCI address (sysfs), or None when unknown."""
    try:
        import torch
        if not torch.cuda.is_available():
            return None
        p = torch.cuda.get_device_properties(torch.cuda.current_device() if device is None else device)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            n = int(f.read().strip())
        return n if n >= 0 else None
    except Exception:
        return None


def numa_cpus(node):
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            return _parse_cpulist(f.read())
    except OSError:
        return []


def rank_cpu_share(local_rank=None, local_world=None, mask=None, online=None, numa=None, ranks_on_node=None):
    """The CPUs this rank's host work should use.

    * A mask narrower than the online CPUs means a launcher (``--bind_cores_to_rank``, taskset,
      Slurm) already bound the rank: keep it.
    * Otherwise the rank takes its slice of its GPU's NUMA node (``numa``: that node's CPUs,
      ``ranks_on_node``: the local ranks whose GPUs share the node, in order) or, with no NUMA
      information, its 1/local_world slice of the host.
    """
    local_rank = _local_rank() if local_rank is None else local_rank
    local_world = _local_world() if local_world is None else local_world
    mask = sorted(os.sched_getaffinity(0) if mask is None else mask)
    online = _online_cpus() if online is None else set(online)
    if len(mask) < len(online):
        return mask, "inherited"
    if numa:
        cand = [c for c in sorted(numa) if c in set(mask)]
        peers = ranks_on_node or [local_rank]
        if cand and local_rank in peers:
            per = max(1, len(cand) // len(peers))
            i = peers.index(local_rank)
            return cand[i * per:(i + 1) * per] or cand[:per], "numa"
    per = max(1, len(mask) // local_world)
    return mask[local_rank * per:(local_rank + 1) * per] or mask[:per], "split"


def host_threads(share, omp_env=None, local_world=None, explicit=None):
    """Thread-team size for the host optimizer: ``SXE_HOST_ADAM_THREADS`` if set; else the rank's CPU
    share, capped by an ``OMP_NUM_THREADS`` above 1 (a deliberate budget, e.g. a shared box). An
    ``OMP_NUM_THREADS=1`` under more than one local rank is torchrun's placeholder, not a budget."""
    explicit = os.environ.get("SXE_HOST_ADAM_THREADS") if explicit is None else explicit
    if explicit:
        return max(1, int(explicit))
    omp_env = os.environ.get("OMP_NUM_THREADS") if omp_env is None else omp_env
    local_world = _local_world() if local_world is None else local_world
    n = max(1, len(share))
    if omp_env:
        try:
            omp = int(omp_env.split(",")[0])
        except ValueError:
            omp = 0
        if omp > 1:
            n = min(n, omp)
        elif omp == 1 and local_world == 1:
            n = 1
    return n


_CONFIGURED = None


def configure_host_threads(bind=None):
    """Size (and, on a GPU host, place) this rank's host-optimizer thread team once per process.
    Returns the thread count. ``bind``: restrict the process affinity to the rank's share so the
    pinned fp32 state is first-touched on the GPU's NUMA node (default on when more than one rank
    shares the host and the process is unbound; ``SXE_HOST_BIND=0`` disables)."""
    global _CONFIGURED
    if _CONFIGURED is not None:
        return _CONFIGURED
    local_world = _local_world()
    node = gpu_numa_node()
    numa = numa_cpus(node) if node is not None else None
    peers = None
    if numa:
        peers = _local_ranks_on_numa(node, local_world)
    share, how = rank_cpu_share(local_world=local_world, numa=numa, ranks_on_node=peers)
    n = host_threads(share, local_world=local_world)
    if bind is None:
        bind = os.environ.get("SXE_HOST_BIND", "1") == "1" and local_world > 1 and how != "inherited"
    if bind:
        try:
            os.sched_setaffinity(0, share)
        except OSError:
            pass
    try:
        import torch
        ops = getattr(torch.ops, "sxe_cpu", None)
        if ops is not None and hasattr(ops, "set_num_threads"):
            ops.set_num_threads(n)
    except Exception:
        pass
    log_dist(f"host optimizer: {n} threads on CPUs {share[0]}-{share[-1]} ({how}"
             f"{f', GPU NUMA node {node}' if node is not None else ''}, {local_world} local ranks"
             f"{', bound' if bind else ''})", ranks=[0])
    _CONFIGURED = n
    return n


def _local_ranks_on_numa(node, local_world):
    """Local ranks whose GPU sits on NUMA node ``node``, assuming local rank i drives visible device i
    (the torchrun / launcher convention)."""
    try:
        import torch
        n = min(local_world, torch.cuda.device_count())
    except Exception:
        return None
    ranks = [r for r in range(n) if gpu_numa_node(r) == node]
    return ranks or None


def mem_available():
    """Host MemAvailable in bytes (None when unknown)."""
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    return int(line.split()[1]) * 1024
    except OSError:
        pass
    return None


def preflight_host_memory(need_bytes, what, local_world=None, available=None, headroom=0.9):
    """Raise before allocating ``need_bytes`` of host memory per rank when the node cannot hold every
    local rank's copy (all ranks of a node allocate the same tier at the same time)."""
    local_world = _local_world() if local_world is None else local_world
    available = mem_available() if available is None else available
    if available is None:
        return
    total = need_bytes * local_world
    if total > headroom * available:
        gib = 2 ** 30
        raise MemoryError(
            f"sxe: {what} needs {need_bytes / gib:.1f} GiB of host memory per rank x {local_world} local ranks = "
            f"{total / gib:.1f} GiB, but the host has {available / gib:.1f} GiB available "
            f"({headroom:.0%} usable). Offload fewer parameters (offload_optimizer.ratio < 1), use "
            f"offload_optimizer.device=nvme, or run more nodes.")
