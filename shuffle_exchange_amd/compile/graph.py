"""Schedule IR of one ZeRO-3 micro-step: the fetch groups in forward order, then in backward order,
each node carrying its measured compute time, its gather size and time, and the live memory when
it starts. This is the graph the passes transform (the reference's counterpart is an FX graph with
``dc.allgather_param`` / ``release_param`` / ``reduce_grad`` nodes, compile/passes/zero3_compile.py)."""
from dataclasses import dataclass, field


@dataclass
class Node:
    phase: str          # "fwd" | "bwd"
    fg: int             # fetch-group index (the ZeRO-3 unit granule)
    compute_ms: float   # compute between this group's fetch and the next event
    live_bytes: int     # device memory (or gathered-parameter bytes) when the node starts


@dataclass
class ScheduleGraph:
    nodes: list
    gather_bytes: dict            # fg -> bytes gathered per fetch (non-persistent units only)
    gather_ms: dict               # fg -> measured (or modelled) all-gather time
    peak_bytes: int               # peak device memory of the traced micro-step
    device_bytes: int             # total device memory
    persistent_bytes: int = 0     # already-persistent unit bytes
    meta: dict = field(default_factory=dict)

    def order(self, phase):
        return [n for n in self.nodes if n.phase == phase]

    def total_compute_ms(self):
        return sum(n.compute_ms for n in self.nodes)

    def summary(self):
        return (f"{len(self.order('fwd'))} fwd / {len(self.order('bwd'))} bwd nodes, "
                f"{sum(self.gather_bytes.values()) / 2**30:.2f} GiB gathered per pass, "
                f"peak {self.peak_bytes / 2**30:.2f} GiB of {self.device_bytes / 2**30:.1f} GiB, "
                f"compute {self.total_compute_ms():.2f} ms")
