"""Schedule passes over a traced ZeRO-3 micro-step (reference compile/passes/: zero3_compile.py,
selective_gather.py, prefetch.py, offload_adam_states.py, offload_activation.py).

Each pass takes the ScheduleGraph, the plan built so far and the memory budget, and returns the
plan. A plan is what stage3.ZeroStage3Optimizer.apply_compile_plan installs:
  keep       fetch groups gathered once and kept resident across steps (re-gathered from the
             updated shards after each optimizer step) -- no per-micro-step all-gather;
  prefetch   {"fwd"|"bwd": {trigger fg: [fgs to start gathering there]}} -- each gather is issued
             far enough ahead to hide behind measured compute, as long as the bytes in flight fit;
  offload_opt_states   park optimizer states on the host during forward/backward;
  offload_activation   keep saved activations in pinned host memory (autograd save_on_cpu).
"""


def zero3_schedule(g, plan, budget):
    """Baseline: gather at first use, release after last use (what the eager hooks do)."""
    plan.setdefault("keep", set())
    plan.setdefault("prefetch", {"fwd": {}, "bwd": {}})
    plan.setdefault("offload_opt_states", False)
    plan.setdefault("offload_activation", False)
    plan.setdefault("log", [])
    return plan


def _headroom(g, plan, budget):
    kept = sum(g.gather_bytes.get(i, 0) for i in plan["keep"])
    return budget - g.peak_bytes - kept


def selective_gather(g, plan, budget):
    """Keep fetch groups resident while the budget allows. Each kept group saves two all-gathers
    per micro-step (forward and backward); the order is by measured gather time per byte, highest
    first -- small groups are latency-bound and cost the most per byte -- then by size."""
    cands = sorted(g.gather_bytes, key=lambda i: (-(g.gather_ms.get(i, 0.0) / max(1, g.gather_bytes[i])),
                                                  g.gather_bytes[i]))
    room = _headroom(g, plan, budget)
    for i in cands:
        b = g.gather_bytes[i]
        if i in plan["keep"] or b > room:
            continue
        plan["keep"].add(i)
        room -= b
    plan["log"].append(f"selective_gather: keep {len(plan['keep'])}/{len(g.gather_bytes)} groups "
                       f"({sum(g.gather_bytes[i] for i in plan['keep']) / 2**30:.2f} GiB)")
    return plan


def prefetch(g, plan, budget, slack=1.25):
    """Place each remaining gather at the latest trigger point whose compute until the group's use
    covers ``slack`` x its measured gather time, moving it later while the bytes in flight at the
    trigger would exceed the headroom (reference prefetch.py's memory-bounded reordering)."""
    room = max(0, _headroom(g, plan, budget))
    out = {"fwd": {}, "bwd": {}}
    issued = 0
    for phase in ("fwd", "bwd"):
        order = g.order(phase)
        inflight = [0] * len(order)  # prefetched bytes outstanding while node k runs
        for k, n in enumerate(order):
            j = n.fg
            if j in plan["keep"] or j not in g.gather_bytes or k == 0:
                continue
            need = slack * g.gather_ms.get(j, 0.0)
            b = g.gather_bytes[j]
            p, acc = k - 1, order[k - 1].compute_ms
            while p > 0 and acc < need and inflight[p - 1] + b <= room:
                p -= 1
                acc += order[p].compute_ms
            while p < k - 1 and any(inflight[q] + b > room for q in range(p, k)):
                p += 1  # memory first: start later
            for q in range(p, k):
                inflight[q] += b
            out[phase].setdefault(order[p].fg, []).append(j)
            issued += 1
    plan["prefetch"] = out
    plan["log"].append(f"prefetch: {issued} gathers scheduled, headroom {room / 2**30:.2f} GiB")
    return plan


def offload_adam_states(g, plan, budget):
    """Park optimizer states on the host during forward/backward when the traced peak (plus what
    selective_gather kept) exceeds the budget (reference offload_adam_states.py)."""
    if _headroom(g, plan, budget) < 0:
        plan["offload_opt_states"] = True
    plan["log"].append(f"offload_adam_states: {plan['offload_opt_states']}")
    return plan


def offload_activation(g, plan, budget):
    """Keep activations saved for backward in pinned host memory when, even after the optimizer
    states leave HBM (their traced bytes credited back), the traced peak exceeds the budget
    (reference offload_activation.py)."""
    over = -_headroom(g, plan, budget)
    if plan.get("offload_opt_states"):
        over -= g.meta.get("optimizer_bytes", 0)
    plan["offload_activation"] = over > 0
    plan["log"].append(f"offload_activation: {plan['offload_activation']}")
    return plan


PASSES = {"zero3_compile": zero3_schedule, "selective_gather": selective_gather, "prefetch": prefetch,
          "offload_adam_states": offload_adam_states, "offload_activation": offload_activation}
