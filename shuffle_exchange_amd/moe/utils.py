"""MoE parameter helpers (parity: reference deepspeed/moe/utils.py:72-182)."""


def is_moe_param(p):
    return hasattr(p, "allreduce") and not p.allreduce


def has_moe_layers(module):
    from .layer import MoE
    for m in module.modules():
        if isinstance(m, MoE):
            return True, m.num_experts
    return False, 0


def split_params_into_different_moe_groups_for_optimizer(param_groups, max_group_size=None):
    """Split every param group into a non-expert group and one group per expert group name
    (``moe=True``, ``name``) so ZeRO can partition/reduce expert params over their own group."""
    if isinstance(param_groups, dict):
        param_groups = [param_groups]
    else:
        param_groups = list(param_groups)
        if param_groups and not isinstance(param_groups[0], dict):
            param_groups = [{"params": param_groups}]
    out = []
    for g in param_groups:
        dense = {**g, "params": [p for p in g["params"] if not is_moe_param(p)]}
        if dense["params"]:
            out.append(dense)
        by_name = {}
        for p in g["params"]:
            if is_moe_param(p):
                by_name.setdefault(p.group_name, []).append(p)
        for name, ps in by_name.items():
            out.append({**g, "params": ps, "moe": True, "name": name})
    return out
