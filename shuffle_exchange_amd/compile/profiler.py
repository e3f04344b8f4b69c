"""Tracing profiler for the schedule compiler (reference compile/profilers/graph_profile.py, which
runs the FX graph node by node and records time and memory).

Here the ZeRO-3 optimizer calls the tracer at its own schedule points -- a fetch group's forward
start (after its gather completed) and end, its backward start, and the end of the micro-step's
backward -- and around every all-gather it launches. On the GPU the points are HIP events
(nothing synchronises until the trace is read) plus ``memory_allocated``; on the CPU (gloo tests)
they are host clocks and the modelled gathered-parameter bytes."""
import time

import torch

from .graph import Node, ScheduleGraph


class ScheduleTracer:
    def __init__(self, opt):
        self.opt = opt
        u0 = next((u for fg in opt.fgroups for u in fg.units), None)
        self.cuda = u0 is not None and u0.flat.is_cuda
        self.complete = None  # the last complete micro-step trace
        self._reset()

    # --------------------------------------------------------------------------------- clocks
    def _now(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def _stamp_on(self, stream):
        if self.cuda and stream is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            return e
        return self._now()

    def _ms(self, a, b):
        return a.elapsed_time(b) if self.cuda else (b - a) * 1e3

    def _live(self):
        if self.cuda:
            return int(torch.cuda.memory_allocated())
        return sum(u.padded * u.flat.element_size() for fg in self.opt.fgroups for u in fg.units
                   if u.state != 0 and u.flat is not None)

    def _reset(self):
        self.events = []     # (phase, fg idx, marker, stamp, live)
        self.gathers = {}    # fg idx -> list of (start, end)
        if self.cuda:
            torch.cuda.reset_peak_memory_stats()

    # ---------------------------------------------------------------------- schedule points
    def on_forward_start(self):
        self._reset()

    def on_fwd_begin(self, fg):
        self.events.append(("fwd", fg.idx, "begin", self._now(), self._live()))

    def on_fwd_end(self, fg):
        self.events.append(("fwd", fg.idx, "end", self._now(), self._live()))

    def on_bwd_begin(self, fg):
        self.events.append(("bwd", fg.idx, "begin", self._now(), self._live()))

    def gather_begin(self, unit, stream):
        return self._stamp_on(stream)

    def gather_end(self, unit, stream, t0):
        self.gathers.setdefault((unit.fg.idx, id(unit)), []).append((t0, self._stamp_on(stream)))

    def on_backward_end(self):
        self.events.append(("bwd", -1, "end", self._now(), self._live()))
        self.complete = (list(self.events), dict(self.gathers),
                         int(torch.cuda.max_memory_allocated()) if self.cuda else max(e[4] for e in self.events))

    # ---------------------------------------------------------------------------- the graph
    def graph(self):
        assert self.complete is not None, "no complete micro-step traced yet"
        events, gathers, peak = self.complete
        if self.cuda:
            torch.cuda.synchronize()
        opt = self.opt
        nodes = []
        fwd = [e for e in events if e[0] == "fwd"]
        for i, e in enumerate(fwd):  # forward: begin -> end of the same group
            if e[2] != "begin":
                continue
            end = next((f for f in fwd[i + 1:] if f[1] == e[1] and f[2] == "end"), None)
            nodes.append(Node("fwd", e[1], self._ms(e[3], end[3]) if end else 0.0, e[4]))
        bwd = [e for e in events if e[0] == "bwd"]
        for i, e in enumerate(bwd):  # backward: begin -> the next backward event
            if e[2] != "begin":
                continue
            nxt = bwd[i + 1] if i + 1 < len(bwd) else None
            nodes.append(Node("bwd", e[1], self._ms(e[3], nxt[3]) if nxt else 0.0, e[4]))
        gb, gm = {}, {}
        for fg in opt.fgroups:
            b = sum(u.padded * u.flat.element_size() for u in fg.units if not u.persistent)
            if b:
                gb[fg.idx] = b
                t = 0.0  # one fetch of the group = one gather of each of its units (mean over fetches)
                for u in fg.units:
                    spans = gathers.get((fg.idx, id(u)))
                    if spans:
                        t += sum(self._ms(a, z) for a, z in spans) / len(spans)
                gm[fg.idx] = t
        persistent = sum(u.padded * u.flat.element_size() for fg in opt.fgroups for u in fg.units if u.persistent)
        dev = torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory if self.cuda else 0
        opt_bytes = sum(t.numel() * t.element_size() for st in getattr(getattr(opt, "optimizer", None), "state", {}).values()
                        for t in st.values() if torch.is_tensor(t) and t.is_cuda)
        return ScheduleGraph(nodes, gb, gm, peak, dev, persistent, meta={"world": opt.S, "optimizer_bytes": opt_bytes})
