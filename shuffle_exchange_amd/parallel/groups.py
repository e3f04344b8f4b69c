"""Process-group registry: data / tensor / pipeline / sequence / expert parallel groups.

Parity: reference deepspeed/utils/groups.py:110-749 (``_get_*_group``, ``_create_expert_and_data_parallel``
:240-440, hpZ ``_create_zero_param_parallel_group`` :692-749) and
runtime/sequence_parallel/parallel_state_sp.py:17-90.

Layout (row-major, last axis fastest): ``[pipe, data, seq, model]``. Tensor parallel is innermost
(largest/most frequent activation all-reduces), then Ulysses sequence parallel (per-layer
all-to-all), then data parallel; pipeline is outermost (lowest-volume p2p). On one 8-GPU MI355X
node every pair is a direct xGMI link, so this order only fixes which ranks share a collective.
ZeRO partitions over the combined (data x seq) group, as the reference does for SP
(``seq_data_parallel_group``, stage_1_and_2.py:1314 divides by dp/sp).
"""
from .. import comm as dist
from .topology import ProcessTopology


class _Registry:
    topo = None
    sizes = dict(tp=1, pp=1, sp=1, dp=1)
    groups = {}
    ranks = {}
    expert = {}  # name -> (ep_group, ep_ranks, edp_group, edp_ranks)
    expert_span = {}  # name -> the EP groups span the TP ranks (no expert TP)
    zero_param = None  # hpZ intra group
    mpu = None


def _make_axis_groups(topo, axis, key):
    me = dist.get_rank()
    mine = None
    for lst in topo.get_axis_comm_lists(axis):
        g = dist.new_group(lst)
        if me in lst:
            mine = (g, lst)
    if mine is None:
        mine = (None, [me])
    _Registry.groups[key], _Registry.ranks[key] = mine


def initialize(tensor_parallel_size=1, pipeline_parallel_size=1, sequence_parallel_size=1, mpu=None):
    """Create every base group once. Safe to call again with the same sizes."""
    W = dist.get_world_size()
    tp, pp, sp = tensor_parallel_size, pipeline_parallel_size, sequence_parallel_size
    assert W % (tp * pp * sp) == 0, f"world {W} not divisible by tp*pp*sp={tp * pp * sp}"
    dp = W // (tp * pp * sp)
    new = dict(tp=tp, pp=pp, sp=sp, dp=dp)
    if _Registry.topo is not None and _Registry.sizes == new and _Registry.mpu is mpu:
        return
    _Registry.mpu = mpu
    _Registry.sizes = new
    _Registry.topo = ProcessTopology(["pipe", "data", "seq", "model"], [pp, dp, sp, tp])
    topo = _Registry.topo
    _Registry.groups, _Registry.ranks, _Registry.expert, _Registry.expert_span = {}, {}, {}, {}
    if mpu is not None:
        _Registry.groups["data"] = mpu.get_data_parallel_group()
        _Registry.ranks["data"] = dist.group_ranks(_Registry.groups["data"])
        _Registry.groups["model"] = mpu.get_model_parallel_group()
        _Registry.ranks["model"] = dist.group_ranks(_Registry.groups["model"])
        _Registry.groups["pipe"], _Registry.ranks["pipe"] = None, [dist.get_rank()]
        _Registry.groups["seq"], _Registry.ranks["seq"] = None, [dist.get_rank()]
        _Registry.groups["seq_data"] = _Registry.groups["data"]
        _Registry.ranks["seq_data"] = _Registry.ranks["data"]
        return
    for axis in ("data", "seq", "model", "pipe"):
        _make_axis_groups(topo, axis, axis)
    # combined (data x seq) group: ranks sharing pipe & model coords
    me = dist.get_rank()
    mine = None
    for p in range(pp):
        for m in range(tp):
            lst = sorted(topo.filter_match(pipe=p, model=m))
            g = dist.new_group(lst)
            if me in lst:
                mine = (g, lst)
    _Registry.groups["seq_data"], _Registry.ranks["seq_data"] = mine


def _ensure():
    if _Registry.topo is None:
        initialize()


def topology():
    _ensure()
    return _Registry.topo


def _g(key):
    _ensure()
    return _Registry.groups.get(key)


def _r(key):
    _ensure()
    return _Registry.ranks.get(key, [dist.get_rank()])


def get_data_parallel_group():
    return _g("data")


def get_data_parallel_world_size():
    return len(_r("data"))


def get_data_parallel_rank():
    return _r("data").index(dist.get_rank())


def get_tensor_model_parallel_group():
    return _g("model")


def get_tensor_model_parallel_world_size():
    return len(_r("model"))


def get_tensor_model_parallel_rank():
    return _r("model").index(dist.get_rank())


def get_pipe_parallel_group():
    return _g("pipe")


def get_pipe_parallel_world_size():
    return len(_r("pipe"))


def get_pipe_parallel_rank():
    return _r("pipe").index(dist.get_rank())


def get_sequence_parallel_group():
    return _g("seq")


def get_sequence_parallel_world_size():
    return len(_r("seq"))


def get_sequence_parallel_rank():
    return _r("seq").index(dist.get_rank())


def get_sequence_data_parallel_group():
    return _g("seq_data")


def get_sequence_data_parallel_world_size():
    return len(_r("seq_data"))


def get_sequence_data_parallel_rank():
    return _r("seq_data").index(dist.get_rank())


def group_ranks(key):
    return list(_r(key))


# ---------------------------------------------------------------------------------------------
# expert parallel (reference utils/groups.py:240-440)
def create_expert_and_data_parallel(ep_size, group_name=None, span_tp=None):
    """Split every data(-x-seq) parallel group into expert-parallel groups of ``ep_size``
    consecutive ranks; expert-data-parallel groups join the ranks holding the same experts.

    ``span_tp`` (tensor parallelism without expert TP; reference groups.py:240
    ``_create_expert_and_data_parallel``, "E + D"): the groups are cut from the whole data x model
    plane of a pipeline stage in rank order, so the ranks of one TP group hold DIFFERENT experts and
    each processes its 1/tp share of the (TP-duplicated) tokens. Without it (the default, and expert
    TP: groups.py:383 ``_create_expert_data_and_model_parallel``, "E + M + D") the groups stay
    inside one TP rank's slice."""
    _ensure()
    name = group_name or f"ep_size_{ep_size}"
    span = bool(span_tp) and _Registry.sizes["tp"] > 1
    if name in _Registry.expert:
        if span_tp is not None and _Registry.expert_span.get(name, False) != span:
            raise ValueError(f"expert group {name} already exists with span_tp={_Registry.expert_span.get(name)}: "
                             "every MoE layer of one ep_size must agree on enable_expert_tensor_parallelism")
        return name
    _Registry.expert_span[name] = span
    topo = _Registry.topo
    me = dist.get_rank()
    sizes = _Registry.sizes
    mine = [None, [me], None, [me]]
    slices = [(p, None) for p in range(sizes["pp"])] if span else \
        [(p, m) for p in range(sizes["pp"]) for m in range(sizes["tp"])]
    for p, m in slices:
        dp_ranks = sorted(topo.filter_match(pipe=p) if m is None else topo.filter_match(pipe=p, model=m))
        n = len(dp_ranks)
        assert n % ep_size == 0, f"data-parallel size {n} not divisible by ep_size {ep_size}"
        for i in range(0, n, ep_size):
            lst = dp_ranks[i:i + ep_size]
            g = dist.new_group(lst)
            if me in lst:
                mine[0], mine[1] = g, lst
        for j in range(ep_size):
            lst = dp_ranks[j::ep_size]
            g = dist.new_group(lst)
            if me in lst:
                mine[2], mine[3] = g, lst
    _Registry.expert[name] = tuple(mine)
    return name


def get_expert_parallel_group(name):
    return _Registry.expert[name][0]


def get_expert_parallel_ranks(name):
    return list(_Registry.expert[name][1])


def get_expert_parallel_world_size(name):
    return len(_Registry.expert[name][1])


def get_expert_parallel_rank(name):
    return _Registry.expert[name][1].index(dist.get_rank())


def get_expert_data_parallel_group(name):
    return _Registry.expert[name][2]


def get_expert_data_parallel_world_size(name):
    return len(_Registry.expert[name][3])


def get_expert_data_parallel_rank(name):
    return _Registry.expert[name][3].index(dist.get_rank())


def get_max_expert_size_name():
    if not _Registry.expert:
        return None
    return max(_Registry.expert, key=lambda k: len(_Registry.expert[k][1]))


def expert_group_names():
    return list(_Registry.expert)


# ---------------------------------------------------------------------------------------------
# hpZ / MiCS secondary partition group (reference utils/groups.py:692-749): consecutive blocks of
# `size` ranks inside the ZeRO group (an 8-GPU xGMI node is the natural block).
def create_zero_param_parallel_group(size):
    _ensure()
    key = f"zero_param_{size}"
    if key in _Registry.groups:
        return _Registry.groups[key]
    ranks = _r("seq_data")
    assert len(ranks) % size == 0
    me = dist.get_rank()
    mine = (None, [me])
    for i in range(0, len(ranks), size):
        lst = ranks[i:i + size]
        g = dist.new_group(lst)
        if me in lst:
            mine = (g, lst)
    _Registry.groups[key], _Registry.ranks[key] = mine
    return mine[0]


def reset():
    _Registry.topo = None
    _Registry.groups, _Registry.ranks, _Registry.expert, _Registry.expert_span = {}, {}, {}, {}


# reference-style private aliases
_get_data_parallel_group = get_data_parallel_group
_get_data_parallel_world_size = get_data_parallel_world_size
_get_data_parallel_rank = get_data_parallel_rank
_get_model_parallel_group = get_tensor_model_parallel_group
_get_sequence_parallel_group = get_sequence_parallel_group
_get_sequence_parallel_world_size = get_sequence_parallel_world_size
_get_sequence_data_parallel_group = get_sequence_data_parallel_group
_get_expert_parallel_group = get_expert_parallel_group
_get_expert_data_parallel_group = get_expert_data_parallel_group
_create_expert_and_data_parallel = create_expert_and_data_parallel
