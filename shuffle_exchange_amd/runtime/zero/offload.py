"""ZeRO-Offload / ZeRO-Infinity: optimizer state and fp32 masters on the host (cpu) or NVMe.

Parity: reference runtime/zero/stage_1_and_2.py cpu_offload paths (:1084-1180, :2094-2110),
stage3.py offload_optimizer / sub-group swapping (:2027-2110), runtime/swap_tensor/
partitioned_optimizer_swapper.py, ops/adam/cpu_adam.py.

MI355X-first choices:
  * gradients are reduced AND accumulated on the GPU in fp32 (one MI355X holds 288 GB; even a 70B
    model's fp32 gradient chunk is 35 GB at dp=8), and cross PCIe ONCE per optimizer step, unit by
    unit on a D2H stream, while the CPU updates the previous unit -- the reference streams partial
    gradients to the host every micro-step;
  * the CPU update is the AVX-512 C++ kernel (csrc/cpu/cpu_adam.cpp) that also writes the bf16
    copy into a pinned buffer, which goes straight back on an H2D stream (for ZeRO-3 with
    offload_param the pinned buffer IS the parameter shard, so nothing is copied back at all);
  * NVMe: per-unit [master | exp_avg | exp_avg_sq] records swapped by the C++ thread-pool AIO
    engine (csrc/cpu/aio.cpp) through a ring of pinned slots: read unit i+1 and write unit i-1
    while unit i updates.
The clip coefficient / overflow flag are computed on the GPU and read once per step (the only host
sync of an offloaded step).
"""
import os

import torch

from ...accelerator import get_accelerator
from ...ops import native
from ...utils.logging import log_dist


HOST_KINDS = ("adam", "lion", "adagrad")  # optimizers with a streamed C++ host kernel


def _pinned(n, dtype):
    return pinned_empty(n, dtype)


def _offsets(units):
    off, out = 0, []
    for u in units:
        out.append(off)
        off += u.chunk
    return out


def pinned_empty(n, dtype):
    """Exact-size pinned host buffer (host_mem.hip) -- the caching host allocator behind
    ``pin_memory=True`` rounds to a power of two, up to +100 % of the host tier's footprint.
    Small buffers and GPU-less processes use the regular path."""
    n = int(n)
    if torch.cuda.is_available() and n * torch.tensor([], dtype=dtype).element_size() >= (64 << 20) \
            and native.hip_available():
        return torch.ops.sxe.pinned_empty(n, dtype)
    return torch.empty(n, dtype=dtype, pin_memory=torch.cuda.is_available())


class _NVMeSwapper:
    """Per parameter group, one file holding every unit's [master | m | v] record (4 KiB aligned)."""

    KINDS = ("master", "exp_avg", "exp_avg_sq")

    def __init__(self, root, rank, units, nkinds, aio_cfg=None, buffer_count=3):
        from ...ops.aio import AsyncIOHandle
        self.dir = os.path.join(root, f"sxe_swap_rank{rank}")
        os.makedirs(self.dir, exist_ok=True)
        a = aio_cfg
        kw = dict(block_size=getattr(a, "block_size", 1 << 20), queue_depth=getattr(a, "queue_depth", 8),
                  intra_op_parallelism=max(2, getattr(a, "intra_op_parallelism", 1) or 1))
        self.rd = AsyncIOHandle(**kw)
        self.wr = AsyncIOHandle(**kw)
        self.nkinds = nkinds
        self.files, self.offsets = [], []
        max_chunk = 1
        for g, us in enumerate(units):
            offs, o = [], 0
            for u in us:
                offs.append(o)
                o += self._rec_bytes(u.chunk)
                max_chunk = max(max_chunk, u.chunk)
            self.files.append(os.path.join(self.dir, f"group{g}.swp"))
            self.offsets.append(offs)
        self.slot_elems = (self._rec_bytes(max_chunk) // 4)
        self.slots = [_pinned(self.slot_elems, torch.float32) for _ in range(max(2, buffer_count))]
        self.slot_write = [None] * len(self.slots)

    def _rec_bytes(self, chunk):
        b = chunk * 4 * self.nkinds
        return (b + 4095) // 4096 * 4096

    def views(self, slot, chunk):
        buf = self.slots[slot]
        return [buf[k * chunk:(k + 1) * chunk] for k in range(self.nkinds)]

    def _rec(self, slot, chunk):
        return self.slots[slot][:self._rec_bytes(chunk) // 4]

    def read(self, slot, g, i, chunk):
        if self.slot_write[slot] is not None:
            self.wr.wait_request(self.slot_write[slot])
            self.slot_write[slot] = None
        return self.rd.async_pread(self._rec(slot, chunk), self.files[g], self.offsets[g][i])

    def write(self, slot, g, i, chunk):
        self.slot_write[slot] = self.wr.async_pwrite(self._rec(slot, chunk), self.files[g], self.offsets[g][i])

    def drain(self):
        self.rd.wait()
        self.wr.wait()
        self.slot_write = [None] * len(self.slots)


class HostOptimizerStep:
    """Plugged into a ZeRO optimizer (``ZeroOptimizerBase.host_step``): owns where the masters and
    the optimizer state live and runs the update there."""

    def __init__(self, offload_config, aio_config=None, rank=0):
        native.require_cpu()
        self.device = offload_config.device
        self.pin = bool(offload_config.pin_memory) or self.device == "nvme"
        self.nvme_path = offload_config.nvme_path
        self.buffer_count = max(3, int(offload_config.buffer_count))
        # Twin-Flow partial offload: the first `ratio` of every param group's elements lives on the
        # host, the rest keeps its masters / state / update in HBM (split_param_groups below)
        self.ratio = float(offload_config.ratio)
        if self.ratio < 1.0 and self.device == "nvme":
            log_dist("offload_optimizer.ratio < 1 applies to device=cpu only: offloading the whole optimizer",
                     ranks=[0])
            self.ratio = 1.0
        self.groups = set()
        self.aio_config = aio_config
        self.rank = rank
        self.swapper = None
        self.materialized = False
        if self.device == "nvme":
            assert self.nvme_path, "offload_optimizer.device=nvme needs nvme_path"
        acc = get_accelerator()
        self.STAGE_SLOTS = max(2, int(os.environ.get("SXE_OFFLOAD_STAGE_SLOTS", 3)))
        self.D2H_PIECE = max(4096, int(os.environ.get("SXE_OFFLOAD_D2H_PIECE", 64 << 20)))  # elements
        self.d2h = acc.named_stream("offload_d2h") if acc.gpu else None
        self.h2d = acc.named_stream("offload_h2d") if acc.gpu else None
        self._h2d_done = None
        # SXE_OFFLOAD_TRACE=1: per-step host timeline of the streamed update (wall time waiting for
        # gradient D2H copies, in the C++ update kernel, waiting for free H2D slots) -- logged and
        # kept in ``self.trace`` (tools/offload_timeline.py turns it into a table)
        self.trace_on = os.environ.get("SXE_OFFLOAD_TRACE", "0") == "1"
        self.trace = []
        # Asynchronous update (SXE_OFFLOAD_ASYNC=1, opt-in; optimizers that declare
        # ``supports_async_host_step``, i.e. ZeRO-3): every unit's gradient crosses PCIe into a pinned
        # host mirror, then a worker thread runs the C++ update unit by unit in the order the next
        # forward needs them and copies each updated bit16 shard back on the H2D stream; step()
        # returns at once and the next forward waits per unit (``wait_units``) instead of for the
        # whole update. Results are bit-identical to the synchronous path (same kernels, same
        # order). Off by default: on the 1-GPU box the forward only waits for the update (the host
        # update is 10x the forward's time) and the worker's OpenMP team ran the update 6-30 %
        # slower than the main thread's, 3,765 vs 4,020 tokens/s on llama70b-infinity
        # (profiles/r05/llama70b-infinity_async_{on,off}.log, timeline
        # llama70b-infinity_async_trace.jsonl).
        self.async_update = os.environ.get("SXE_OFFLOAD_ASYNC", "0") == "1" and self.device == "cpu"
        # asynchronous tier, copy scheduling: SXE_OFFLOAD_ASYNC_WINDOW=W > 0 keeps only W units' gradient
        # D2H copies queued ahead of the host update (the worker issues unit k + W's when unit k is done)
        # instead of the whole mirror at step() -- an updated shard's H2D then queues behind at most W
        # D2H pieces on the copy engine; SXE_OFFLOAD_H2D_KERNEL=1 moves the updated shards with a kernel
        # that reads the pinned buffer over the link (host_mem.hip h2d_copy_), off the copy engines
        self.async_window = int(os.environ.get("SXE_OFFLOAD_ASYNC_WINDOW", "0"))
        self.h2d_kernel = os.environ.get("SXE_OFFLOAD_H2D_KERNEL", "0") == "1"
        self._worker = None
        self._ready = {}
        self._h2d_ev = {}
        self._pending = False
        self._error = None
        self.ghost = None

    # ------------------------------------------------------------------------------------ layout
    def _kinds(self, opt):
        return {"adam": 3, "lion": 2, "adagrad": 2}.get(opt.kind, 1)

    def host_groups(self, opt):
        """Indices of the param groups this tier owns (all of them unless Twin-Flow split them)."""
        return {g for g, pg in enumerate(opt.optimizer.param_groups) if pg.get("sxe_offload", True)}

    def init_master(self, opt):
        if opt.kind not in HOST_KINDS and self.device == "nvme":
            raise ValueError("NVMe optimizer offload supports Adam/AdamW/Lion/Adagrad")
        self.groups = self.host_groups(opt)
        self._preflight(opt)
        G = len(opt.units)
        opt.grad_host, opt.lp_host = [None] * G, [None] * G
        # Host staging of gradients (fp32, D2H) and updated bit16 params (H2D): a ring of
        # STAGE_SLOTS unit-sized pinned slots instead of full-model mirrors (6 B/param less on the
        # host -- the host tier is what bounds the trainable model size); generic torch optimizers
        # step whole groups and keep the full mirrors.
        self.streamed = opt.kind in HOST_KINDS  # C++ CPU kernels; others step torch-side on mirrors
        all_units = [u for g in sorted(self.groups) for u in opt.units[g]]
        if self.streamed and all_units:
            maxc = max(u.chunk for u in all_units)
            self.gslots = [_pinned(maxc, torch.float32) for _ in range(self.STAGE_SLOTS)]
            lp_dtype = next((u.dtype for u in all_units if u.shard_is_cuda()), None)
            self.lslots = [_pinned(maxc, lp_dtype) for _ in range(self.STAGE_SLOTS)] if lp_dtype else None
            self._lslot_ev = [None] * self.STAGE_SLOTS
        for g, units in enumerate(opt.units):
            if g not in self.groups:
                continue  # Twin-Flow device group: initialised by the ZeRO optimizer itself
            total = sum(u.chunk for u in units)
            gr = torch.zeros(total, dtype=torch.float32, device=opt.device)  # GPU accumulator
            needs_lp = any(u.shard_is_cuda() for u in units)
            opt.grad_host[g] = None if self.streamed else _pinned(total, torch.float32)
            opt.lp_host[g] = _pinned(total, units[0].dtype) if needs_lp and not self.streamed else None
            if self.device == "cpu":
                m = _pinned(total, torch.float32) if self.pin else torch.empty(total, dtype=torch.float32)
            else:
                m = torch.empty(0, dtype=torch.float32)
            off = 0
            for u in units:
                u.grad = gr[off:off + u.chunk]
                if self.device == "cpu":
                    u.master = m[off:off + u.chunk]
                    u.master.copy_(u.shard.float().cpu() if u.shard.is_cuda else u.shard.float())
                else:
                    u.master = None
                off += u.chunk
            m = torch.nn.Parameter(m, requires_grad=False)
            opt.master[g] = m
            opt.grads[g] = gr
            opt.optimizer.param_groups[g]["params"] = [m]
        opt.optimizer.state.clear()
        if self.device == "cpu":
            opt._init_state()
            return
        self.swapper = _NVMeSwapper(self.nvme_path, self.rank, opt.units, self._kinds(opt), self.aio_config,
                                    self.buffer_count)
        for g, units in enumerate(opt.units):
            st = opt.optimizer.state[opt.master[g]]
            st["step"] = 0
            for i, u in enumerate(units):
                views = self.swapper.views(0, u.chunk)
                views[0].copy_(u.shard.float().cpu() if u.shard.is_cuda else u.shard.float())
                for v in views[1:]:
                    v.zero_()
                self.swapper.write(0, g, i, u.chunk)
                self.swapper.drain()
        log_dist(f"ZeRO-Infinity: optimizer state on NVMe under {self.swapper.dir}", ranks=[0])

    def _preflight(self, opt):
        """Host bytes this rank's tier allocates, checked against the node's MemAvailable for every
        local rank before the first allocation (a 70B model offloaded by 8 ranks needs ~1 TB)."""
        from ...utils.host_resources import configure_host_threads, preflight_host_memory
        self.threads = configure_host_threads()
        units = [u for g in sorted(self.groups) for u in opt.units[g]]
        if not units:
            return
        total = sum(u.chunk for u in units)
        maxc = max(u.chunk for u in units)
        streamed = opt.kind in HOST_KINDS
        per_elem = (4 * self._kinds(opt)) if self.device == "cpu" else 0  # master + optimizer states
        if not streamed:
            per_elem += 4 + 2  # full-group gradient and bit16 mirrors
        slots = self.STAGE_SLOTS * maxc * 6 if streamed else 0
        if self.device == "nvme":
            slots += self.buffer_count * maxc * 4 * self._kinds(opt)
        preflight_host_memory(total * per_elem + slots,
                              f"ZeRO-Offload optimizer tier ({self.device}, {total / 1e9:.2f} G elements)")

    # ------------------------------------------------------------------------------------ update
    def _host_kernel(self, opt, pg, st, master, grad, states, lp, coef):
        ops = torch.ops.sxe_cpu
        if opt.kind == "adam":
            b1, b2 = pg["betas"]
            fused_lp = lp if (lp is not None and lp.dtype in (torch.bfloat16, torch.float16)) else None
            ops.adam_step_(master, grad, states[0], states[1], fused_lp, float(pg["lr"]), float(b1), float(b2),
                           float(pg["eps"]), float(pg["weight_decay"]), int(st["step"]), bool(opt.adamw),
                           bool(pg.get("bias_correction", True)), coef)
            if lp is not None and fused_lp is None:
                lp.copy_(master)
        elif opt.kind == "lion":
            b1, b2 = pg["betas"]
            grad.mul_(coef)
            ops.lion_step_(master, grad, states[0], float(pg["lr"]), float(b1), float(b2), float(pg["weight_decay"]))
            if lp is not None:
                lp.copy_(master)
        elif opt.kind == "adagrad":
            grad.mul_(coef)
            ops.adagrad_step_(master, grad, states[0], float(pg["lr"]), float(pg.get("eps", 1e-10)),
                              float(pg.get("weight_decay", 0.0)))
            if lp is not None:
                lp.copy_(master)

    def _state_views(self, opt, g, o, n):
        st = opt.optimizer.state[opt.master[g]]
        if opt.kind == "adam":
            return [st["exp_avg"][o:o + n], st["exp_avg_sq"][o:o + n]]
        if opt.kind == "lion":
            return [st["exp_avg"][o:o + n]]
        if opt.kind == "adagrad":
            return [st["sum"][o:o + n]]
        return []

    def update(self, opt, coef_t, skip_t):
        if not self.groups:
            return  # Twin-Flow ratio 0: everything is stepped in device memory
        flags = torch.cat([coef_t.reshape(1).float(), skip_t.reshape(1).float()]).cpu()  # the one sync
        coef, skip = float(flags[0]), float(flags[1])
        if skip != 0.0:
            return
        if self.materialized and self.device == "nvme":
            self.flush(opt)
        cur = torch.cuda.current_stream() if opt.device is not None and opt.device.type == "cuda" else None
        if not self.streamed:
            return self._update_mirrored(opt, cur, coef)
        # units in step order; unit k's gradient lands in staging slot k % NS, so at most NS units'
        # copies are in flight ahead of the CPU update
        flat = [(g, i, u, off) for g, units in enumerate(opt.units) if g in self.groups
                for i, u, off in zip(range(len(units)), units, _offsets(units))]
        if self._async_ok(opt, flat):
            return self._update_async(opt, cur, coef, flat)
        NS = len(self.gslots)
        d2h_ev = {}
        # Each unit's gradient crosses in PIECE-element pieces with an event per piece, and the C++
        # update walks the pieces as they land: the CPU no longer waits for a whole unit's copy (74 ms
        # per step for the first, 1 G-element unit of Llama-3-70B) before it can start.
        PIECE = self.D2H_PIECE
        import time as _time
        tr = {"t0": _time.perf_counter(), "d2h_wait": 0.0, "cpu": 0.0, "h2d_wait": 0.0, "units": len(flat),
              "elems": sum(x[2].chunk for x in flat)} if self.trace_on else None

        def issue_d2h(k):
            u = flat[k][2]
            dst = self.gslots[k % NS][:u.chunk]
            if cur is None:
                dst.copy_(u.grad)
                return
            evs = []
            with get_accelerator().stream(self.d2h):
                for a in range(0, u.chunk, PIECE):
                    b = min(u.chunk, a + PIECE)
                    dst[a:b].copy_(u.grad[a:b], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.d2h)
                    evs.append((a, b, ev))
            d2h_ev[k] = evs

        if cur is not None:
            self.d2h.wait_stream(cur)
        for k in range(min(NS, len(flat))):
            issue_d2h(k)
        nvme = self.device == "nvme"
        nslot = len(self.swapper.slots) if nvme else 0
        for g in self.groups:
            st = opt.optimizer.state[opt.master[g]]
            if opt.kind in ("adam", "adagrad"):
                st["step"] = int(st.get("step", 0)) + 1
        pend = {}
        if nvme and flat:
            g0, i0, u0, _ = flat[0]
            pend[0] = self.swapper.read(0, g0, i0, u0.chunk)
        for k, (g, i, u, off) in enumerate(flat):
            pg = opt.optimizer.param_groups[g]
            st = opt.optimizer.state[opt.master[g]]
            if nvme and k + 1 < len(flat):
                gn, iN, un, _ = flat[k + 1]
                pend[k + 1] = self.swapper.read((k + 1) % nslot, gn, iN, un.chunk)
            pieces = d2h_ev.pop(k, None) or [(0, u.chunk, None)]
            slot = k % NS
            grad = self.gslots[slot][:u.chunk]
            if nvme:
                self.swapper.rd.wait_request(pend.pop(k))
                views = self.swapper.views(k % nslot, u.chunk)
                master, states = views[0], views[1:]
            else:
                master, states = u.master, self._state_views(opt, g, off, u.chunk)
            if u.shard_is_cuda():
                if self._lslot_ev[slot] is not None:
                    if tr is not None:
                        t = _time.perf_counter()
                    self._lslot_ev[slot].synchronize()  # its previous H2D has drained
                    if tr is not None:
                        tr["h2d_wait"] += _time.perf_counter() - t
                lp = self.lslots[slot][:u.chunk]
            else:
                lp = u.shard_for_overwrite()  # pinned host shard, or an NVMe swap buffer
            for a, b, ev in pieces:
                if ev is not None:
                    if tr is not None:
                        t = _time.perf_counter()
                    ev.synchronize()
                    if tr is not None:
                        tr["d2h_wait"] += _time.perf_counter() - t
                if tr is not None:
                    t = _time.perf_counter()
                if a == 0 and b == u.chunk:
                    self._host_kernel(opt, pg, st, master, grad, states, lp, coef)
                else:
                    self._host_kernel(opt, pg, st, master[a:b], grad[a:b], [x[a:b] for x in states], lp[a:b], coef)
                if tr is not None:
                    tr["cpu"] += _time.perf_counter() - t
            if nvme:
                self.swapper.write(k % nslot, g, i, u.chunk)
            if k + NS < len(flat):
                issue_d2h(k + NS)  # this grad slot is free again
            if u.shard_is_cuda():
                with get_accelerator().stream(self.h2d):
                    u.shard.copy_(lp, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.h2d)
                    self._lslot_ev[slot] = ev
        if nvme:
            self.swapper.drain()
        if getattr(opt, "pswap", None) is not None:
            opt.pswap.flush()  # updated NVMe-tier shards back to their swap file
        if cur is not None:
            cur.wait_stream(self.d2h)  # zero_grad_buffers() must not overtake the copies
            cur.wait_stream(self.h2d)
        if tr is not None:
            if cur is not None:
                torch.cuda.synchronize()
            tr["wall"] = _time.perf_counter() - tr["t0"]
            tr["threads"] = int(torch.ops.sxe_cpu.num_threads())
            self.trace.append(tr)
            gb = tr["elems"] * 4 / 1e9
            log_dist(f"offload step: wall {tr['wall'] * 1e3:.0f} ms | C++ update {tr['cpu'] * 1e3:.0f} ms "
                     f"({gb * 4 / max(tr['cpu'], 1e-9):.0f} GB/s of fp32 state) | waiting on grad D2H "
                     f"{tr['d2h_wait'] * 1e3:.0f} ms | waiting on H2D slots {tr['h2d_wait'] * 1e3:.0f} ms | "
                     f"{tr['units']} units, {tr['elems'] / 1e9:.2f} G elements, {tr['threads']} threads", ranks=[0])

    # ------------------------------------------------------------------------ asynchronous update
    def _async_ok(self, opt, flat):
        if not (self.async_update and flat and getattr(opt, "supports_async_host_step", False)):
            return False
        if getattr(opt, "pswap", None) is not None:
            return False  # NVMe parameter tier: its swap buffers are driven from the main thread
        if self.ghost is not None:
            return True
        need = sum(x[2].chunk for x in flat) * 4
        try:
            import psutil
            avail = psutil.virtual_memory().available
        except Exception:
            return False
        if need > avail // 2:  # the mirror must leave the host room: else stream through the slot ring
            log_dist(f"offload: {need / 2**30:.1f} GiB gradient mirror does not fit host memory; "
                     "synchronous host update", ranks=[0])
            self.async_update = False
            return False
        return True

    def _update_async(self, opt, cur, coef, flat):
        import threading
        import time as _time
        self.wait_all()
        order = getattr(opt, "host_unit_order", None)
        if order is not None:  # the next forward's order: its first units are ready first
            rank = {id(u): r for r, u in enumerate(order())}
            flat = sorted(flat, key=lambda x: rank.get(id(x[2]), len(rank)))
        total = sum(x[2].chunk for x in flat)
        if self.ghost is None or self.ghost.numel() < total:
            self.ghost = _pinned(total, torch.float32)
        t0 = _time.perf_counter()
        if cur is not None:
            self.d2h.wait_stream(cur)
            self._grads_ready = torch.cuda.Event()  # the backward that wrote u.grad (windowed issue)
            self._grads_ready.record(cur)
        d2h, o = [], 0
        for g, i, u, off in flat:
            d2h.append([self.ghost[o:o + u.chunk], None])
            o += u.chunk
        window = self.async_window if (self.async_window > 0 and cur is not None) else len(flat)

        PIECE = self.D2H_PIECE

        def issue(k):
            # the unit's gradient crosses in PIECE-element pieces with an event per piece; the worker's
            # C++ update walks the pieces as they land (as the synchronous tier does) instead of
            # waiting for the whole unit's copy
            dst, u = d2h[k][0], flat[k][2]
            if cur is None:
                dst.copy_(u.grad)
                return
            evs = []
            with get_accelerator().stream(self.d2h):
                for a in range(0, u.chunk, PIECE):
                    b = min(u.chunk, a + PIECE)
                    dst[a:b].copy_(u.grad[a:b], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.d2h)
                    evs.append((a, b, ev))
            d2h[k][1] = evs
        self._issued_all = threading.Event()
        for k in range(min(window, len(flat))):
            issue(k)
        if window >= len(flat):
            self._issued_all.set()
        # Invariant: nothing may write u.grad on the compute stream until these copies have read it.
        # The compute stream is NOT made to wait here (that would serialise the next forward behind the
        # mirror); every writer of the accumulators calls wait_grad_mirror() / before_backward() first
        # -- which, with a windowed issue, also wait until the worker has issued every copy.
        self._d2h_last = (d2h, len(flat) - 1) if flat else None
        for g in self.groups:
            st = opt.optimizer.state[opt.master[g]]
            if opt.kind in ("adam", "adagrad"):
                st["step"] = int(st.get("step", 0)) + 1
        self._ready = {id(x[2]): threading.Event() for x in flat}
        self._h2d_ev = {}
        self._error = None
        self._pending = True
        tr = {"t0": t0, "units": [], "waits": [], "elems": total} if self.trace_on else None
        self._cur_trace = tr
        dev = opt.device if cur is not None else None

        def work():
            try:
                if dev is not None:
                    torch.cuda.set_device(dev)
                cops = getattr(torch.ops, "sxe_cpu", None)
                if cops is not None and hasattr(cops, "set_num_threads"):
                    # one CPU stays with the training thread, which keeps launching the next
                    # forward's kernels while this team updates (per-thread OpenMP setting: a new
                    # thread starts from the env default, so pass the rank's share explicitly)
                    n = getattr(self, "threads", None) or int(cops.num_threads())
                    cops.set_num_threads(max(1, int(n) - 1))
                NS = len(self.gslots)
                for k, (g, i, u, off) in enumerate(flat):
                    grad, evs = d2h[k]
                    ta = _time.perf_counter()
                    pg = opt.optimizer.param_groups[g]
                    st = opt.optimizer.state[opt.master[g]]
                    slot = k % NS
                    if u.shard_is_cuda():
                        if self._lslot_ev[slot] is not None:
                            self._lslot_ev[slot].synchronize()  # its previous H2D has drained
                        lp = self.lslots[slot][:u.chunk]
                    else:
                        lp = u.shard_for_overwrite()
                    states = self._state_views(opt, g, off, u.chunk)
                    wait = 0.0
                    for a, b, ev in (evs if evs is not None else [(0, u.chunk, None)]):
                        tw = _time.perf_counter()
                        if ev is not None:
                            ev.synchronize()
                        wait += _time.perf_counter() - tw
                        if a == 0 and b == u.chunk:
                            self._host_kernel(opt, pg, st, u.master, grad, states, lp, coef)
                        else:
                            self._host_kernel(opt, pg, st, u.master[a:b], grad[a:b], [x[a:b] for x in states],
                                              lp[a:b], coef)
                    tb = ta + wait
                    tc = _time.perf_counter()
                    if u.shard_is_cuda():
                        with get_accelerator().stream(self.h2d):
                            if self.h2d_kernel and (u.chunk * lp.element_size()) % 16 == 0:
                                torch.ops.sxe.h2d_copy_(u.shard, lp)
                            else:
                                u.shard.copy_(lp, non_blocking=True)
                            hev = torch.cuda.Event()
                            hev.record(self.h2d)
                        self._lslot_ev[slot] = hev
                        self._h2d_ev[id(u)] = hev
                    if k + window < len(flat):
                        if k == 0 and cur is not None:
                            self.d2h.wait_event(self._grads_ready)
                        issue(k + window)
                        if k + window == len(flat) - 1:
                            self._issued_all.set()
                    if tr is not None:
                        tr["units"].append((u.name, u.chunk, ta - t0, tb - t0, tc - t0))
                    self._ready[id(u)].set()
            except BaseException as e:  # surfaced by wait_unit / wait_all on the main thread
                self._error = e
                for e2 in self._ready.values():
                    e2.set()
                self._issued_all.set()

        self._worker = threading.Thread(target=work, name="sxe-host-adam", daemon=True)
        self._worker.start()
        if not getattr(self, "_atexit_set", False):
            # a process that ends while the worker is inside the C++ update (OpenMP team running)
            # aborts in the runtime's teardown ("terminate called without an active exception"):
            # join it first
            import atexit
            import weakref
            ref = weakref.ref(self)
            atexit.register(lambda: ref() is not None and ref()._join_worker())
            self._atexit_set = True

    def _join_worker(self):
        w = self._worker
        if w is not None:
            w.join()

    def _raise(self):
        if self._error is not None:
            e, self._error = self._error, None
            raise RuntimeError("host optimizer update failed") from e

    def wait_unit(self, u):
        """The calling stream may read unit ``u``'s bit16 shard (async update finished for it)."""
        if not self._pending:
            return
        ev = self._ready.get(id(u))
        if ev is None:
            return
        if not ev.is_set():
            import time as _time
            t = _time.perf_counter()
            ev.wait()
            tr = getattr(self, "_cur_trace", None)
            if tr is not None:
                tr["waits"].append((u.name, t - tr["t0"], _time.perf_counter() - tr["t0"]))
        self._raise()
        h = self._h2d_ev.get(id(u))
        if h is not None:
            torch.cuda.current_stream().wait_event(h)

    def wait_units(self, units):
        for u in units:
            self.wait_unit(u)

    def wait_all(self):
        """Finish the asynchronous update: every shard final, the compute stream ordered after it."""
        if self._worker is not None:
            self._worker.join()
            self._worker = None
        self._raise()
        if self._pending:
            if self.h2d is not None and torch.cuda.is_available():
                torch.cuda.current_stream().wait_stream(self.h2d)
            self._pending = False
            tr = getattr(self, "_cur_trace", None)
            if tr is not None and tr["units"]:
                self._log_async_trace(tr)
                self._cur_trace = None

    def before_backward(self):
        """The backward rewrites the fp32 gradient accumulators: the D2H copies of the previous
        asynchronous update must have read them (all of them issued first, with a windowed issue)."""
        ia = getattr(self, "_issued_all", None)
        if ia is not None:
            ia.wait()
        self._raise_if_failed()
        if self.d2h is not None and torch.cuda.is_available():
            torch.cuda.current_stream().wait_stream(self.d2h)

    def _raise_if_failed(self):
        if getattr(self, "_error", None) is not None:
            self.wait_all()

    def wait_grad_mirror(self):
        """Order the current stream after the last gradient-mirror D2H copy of the pending asynchronous
        update (a no-op once it has been waited for). Call before any eager write of ``u.grad``."""
        last = getattr(self, "_d2h_last", None)
        if last is None:
            return
        ia = getattr(self, "_issued_all", None)
        if ia is not None:
            ia.wait()
        d2h, k = last
        evs = d2h[k][1]
        ev = evs[-1][2] if evs else None
        if ev is not None and torch.cuda.is_available():
            torch.cuda.current_stream().wait_event(ev)
        self._d2h_last = None

    def _log_async_trace(self, tr):
        self.trace.append(tr)
        path = os.environ.get("SXE_OFFLOAD_TRACE_FILE")
        if path and self.rank == 0:  # host timeline of every step, JSON lines (tools/offload_timeline.py)
            import json
            with open(path, "a") as f:
                f.write(json.dumps({"units": tr["units"], "waits": tr["waits"], "elems": tr["elems"]}) + "\n")
        last = tr["units"][-1]
        cpu = sum(c - b for _, _, _, b, c in tr["units"])
        d2h_wait = sum(b - a for _, _, a, b, _ in tr["units"])
        fwd_wait = sum(b - a for _, a, b in tr["waits"])
        log_dist(f"offload async step: host update done at {last[4] * 1e3:.0f} ms | C++ update {cpu * 1e3:.0f} ms "
                 f"({tr['elems'] * 16 / 1e9 / max(cpu, 1e-9):.0f} GB/s of fp32 state) | worker waiting on grad D2H "
                 f"{d2h_wait * 1e3:.0f} ms | next forward waited {fwd_wait * 1e3:.0f} ms on {len(tr['waits'])} units",
                 ranks=[0])

    def _update_mirrored(self, opt, cur, coef):
        """Generic (torch) optimizers: full host mirrors of grads / bit16 params."""
        if self._h2d_done is not None:
            self._h2d_done.synchronize()  # lp_host of the previous step fully consumed
        events = []
        if cur is not None:
            self.d2h.wait_stream(cur)
        with get_accelerator().stream(self.d2h):
            for g, units in enumerate(opt.units):
                off = 0
                for u in units:
                    opt.grad_host[g][off:off + u.chunk].copy_(u.grad, non_blocking=True)
                    off += u.chunk
                    if cur is not None:
                        ev = torch.cuda.Event()
                        ev.record(self.d2h)
                        events.append(ev)
        if cur is not None:
            cur.wait_stream(self.d2h)
        k = 0
        for g, units in enumerate(opt.units):
            self._generic(opt, g, events, k, coef)
            k += len(units)
        if cur is not None:
            self._h2d_done = torch.cuda.Event()
            self._h2d_done.record(self.h2d)
            cur.wait_stream(self.h2d)

    def _generic(self, opt, g, events, k, coef):
        units = opt.units[g]
        for j in range(len(units)):
            if events:
                events[k + j].synchronize()
        m = opt.master[g]
        m.grad = opt.grad_host[g] * coef
        # step only this group's params
        saved = [pg["params"] for pg in opt.optimizer.param_groups]
        for j, pg in enumerate(opt.optimizer.param_groups):
            pg["params"] = saved[j] if j == g else []
        opt.optimizer.step()
        for j, pg in enumerate(opt.optimizer.param_groups):
            pg["params"] = saved[j]
        m.grad = None
        off = 0
        for u in units:
            if u.shard_is_cuda():
                lp = opt.lp_host[g][off:off + u.chunk]
                lp.copy_(u.master)
                with get_accelerator().stream(self.h2d):
                    u.shard.copy_(lp, non_blocking=True)
            else:
                u.shard_for_overwrite().copy_(u.master)
            off += u.chunk
        if getattr(opt, "pswap", None) is not None:
            opt.pswap.flush()

    # ------------------------------------------------------------------------- checkpoint support
    def materialize(self, opt):
        """NVMe: read every record into full host tensors (master + optimizer state) so the usual
        state_dict() sees them. No-op for cpu offload (beyond finishing an asynchronous update)."""
        self.wait_all()
        if self.device != "nvme" or self.materialized:
            return
        sw = self.swapper
        for g, units in enumerate(opt.units):
            total = sum(u.chunk for u in units)
            full = [torch.empty(total, dtype=torch.float32) for _ in range(sw.nkinds)]
            off = 0
            for i, u in enumerate(units):
                sw.rd.wait_request(sw.read(0, g, i, u.chunk))
                for dst, src in zip(full, sw.views(0, u.chunk)):
                    dst[off:off + u.chunk].copy_(src)
                u.master = full[0][off:off + u.chunk]
                off += u.chunk
            opt.master[g].data = full[0]
            st = opt.optimizer.state[opt.master[g]]
            names = {"adam": ["exp_avg", "exp_avg_sq"], "lion": ["exp_avg"], "adagrad": ["sum"]}[opt.kind]
            for name, t in zip(names, full[1:]):
                st[name] = t
        self.materialized = True

    def flush(self, opt):
        """NVMe: write materialized host tensors back to the swap files and drop them."""
        if self.device != "nvme":
            return
        sw = self.swapper
        names = {"adam": ["exp_avg", "exp_avg_sq"], "lion": ["exp_avg"], "adagrad": ["sum"]}[opt.kind]
        for g, units in enumerate(opt.units):
            st = opt.optimizer.state[opt.master[g]]
            full = [opt.master[g].data] + [st[n] for n in names]
            off = 0
            for i, u in enumerate(units):
                for dst, src in zip(sw.views(0, u.chunk), full):
                    dst.copy_(src[off:off + u.chunk])
                sw.write(0, g, i, u.chunk)
                sw.drain()
                u.master = None
                off += u.chunk
            opt.master[g].data = torch.empty(0, dtype=torch.float32)
            for n in names:
                st.pop(n, None)
        self.materialized = False

    def write_master(self, opt, u):
        """After an external edit of a unit's bit16 shard: refresh its fp32 master."""
        self.wait_all()
        if self.device == "cpu":
            u.master.copy_(u.shard.float().cpu() if u.shard.is_cuda else u.shard.float())
            return
        g = next(i for i, us in enumerate(opt.units) if any(x is u for x in us))
        i = next(j for j, x in enumerate(opt.units[g]) if x is u)
        sw = self.swapper
        sw.rd.wait_request(sw.read(0, g, i, u.chunk))
        sw.views(0, u.chunk)[0].copy_(u.shard.float().cpu() if u.shard.is_cuda else u.shard.float())
        sw.write(0, g, i, u.chunk)
        sw.drain()


def split_param_groups(optimizer, ratio):
    """Twin-Flow partial offload (reference runtime/zero/stage3.py:867-876 puts the first
    int(ratio * n) optimizer sub-groups on the CPU, the rest on the accelerator): every param group
    is cut, in parameter order, into a host part -- the parameters starting within the first
    ``ratio`` of the group's elements -- and a device part. Both parts keep the group's
    hyper-parameters (LR schedules and clipping see them as ordinary groups) and carry the
    ``sxe_offload`` tag that ``HostOptimizerStep.host_groups`` reads. The device part's masters,
    Adam moments and update stay in HBM (fused HIP Adam), so HBM holds 6 + 12 (1 - ratio) bytes per
    trainable parameter and the host 12 ratio + staging: the ratio trades host RAM for HBM."""
    ratio = min(max(float(ratio), 0.0), 1.0)
    out, origin = [], []
    for gi, pg in enumerate(optimizer.param_groups):
        params = list(pg["params"])
        total = sum(p.numel() for p in params)
        host, dev, start = [], [], 0
        for p in params:
            (host if start < ratio * total else dev).append(p)
            start += p.numel()
        for part, flag in ((host, True), (dev, False)):
            if part:
                out.append(dict(pg, params=part, sxe_offload=flag))
                origin.append(gi)
    n_orig = len(optimizer.param_groups)
    optimizer.param_groups[:] = out
    optimizer._sxe_group_origin = (n_orig, origin)
    return optimizer


def expand_scheduler_groups(scheduler, optimizer):
    """A client LR scheduler built before ``split_param_groups`` holds one entry per ORIGINAL
    param group (``base_lrs``, ``_last_lr``, ``lr_lambdas`` ...): expand every such per-group list to
    the split groups, so both parts of a group follow the group's schedule."""
    info = getattr(optimizer, "_sxe_group_origin", None)
    if info is None or scheduler is None:
        return scheduler
    n_orig, origin = info
    if getattr(scheduler, "optimizer", None) is not None:
        scheduler.optimizer = optimizer
    for k, v in list(vars(scheduler).items()):
        if isinstance(v, list) and len(v) == n_orig and k != "optimizer":
            setattr(scheduler, k, [v[i] for i in origin])
    return scheduler


def OffloadOptimizer(*a, **kw):  # pragma: no cover - kept for the reference's class name
    raise TypeError("use HostOptimizerStep via the engine's zero_optimization.offload_optimizer config")
