"""Cartesian process topology (parity: reference runtime/pipe/topology.py:12 ProcessTopology,
:232 PipeDataParallelTopology, :244 PipeModelDataParallelTopology, :251 PipelineParallelGrid).

Ranks are laid out row-major over the axes, last axis fastest. On one MI355X node every GPU pair is
one xGMI hop, so the placement rule is about collective *sizes*: the axis with the largest and most
frequent traffic (tensor parallel) is innermost, pipeline outermost.
"""
from collections import namedtuple
from itertools import product


class ProcessTopology:
    def __init__(self, axes, dims):
        assert len(axes) == len(dims)
        self.axes = list(axes)
        self.dims = list(dims)
        self.ProcessCoord = namedtuple("ProcessCoord", axes)
        self.mapping = {}
        for rank, coord in enumerate(product(*[range(d) for d in dims])):
            self.mapping[self.ProcessCoord(*coord)] = rank

    def get_rank(self, **coord):
        key = self.ProcessCoord(**coord)
        return self.mapping[key]

    def get_axis_names(self):
        return self.axes

    def get_rank_repr(self, rank, omit_axes=("data", "pipe"), inner_sep="_", outer_sep="-"):
        coord = self.get_coord(rank)
        parts = [f"{a}{inner_sep}{getattr(coord, a):02d}" for a in self.axes if a not in omit_axes]
        return outer_sep.join(parts)

    def get_dim(self, axis):
        return self.dims[self.axes.index(axis)] if axis in self.axes else 1

    def get_coord(self, rank):
        for c, r in self.mapping.items():
            if r == rank:
                return c
        raise ValueError(f"rank {rank} not in topology")

    def get_axis_comm_lists(self, axis):
        """Lists of ranks that differ only along `axis` (one communicator each)."""
        if axis not in self.axes:
            return []
        others = [a for a in self.axes if a != axis]
        lists = []
        for oc in product(*[range(self.get_dim(a)) for a in others]):
            fixed = dict(zip(others, oc))
            lists.append([self.get_rank(**fixed, **{axis: i}) for i in range(self.get_dim(axis))])
        return lists

    def filter_match(self, **filter_kwargs):
        return [r for c, r in self.mapping.items() if all(getattr(c, k) == v for k, v in filter_kwargs.items())]

    def get_axis_list(self, axis, idx):
        ai = self.axes.index(axis)
        return sorted(r for c, r in self.mapping.items() if c[ai] == idx)

    def world_size(self):
        n = 1
        for d in self.dims:
            n *= d
        return n

    def __str__(self):
        return str(self.mapping)


class PipeDataParallelTopology(ProcessTopology):
    def __init__(self, num_pp, num_dp):
        super().__init__(axes=["pipe", "data"], dims=[num_pp, num_dp])


class PipeModelDataParallelTopology(ProcessTopology):
    def __init__(self, num_pp, num_mp, num_dp):
        super().__init__(axes=["pipe", "data", "model"], dims=[num_pp, num_dp, num_mp])


class PipelineParallelGrid:
    """Groups for a (pipe, data[, model]) topology, created once (reference topology.py:251)."""

    def __init__(self, topology=None, process_group=None):
        from .. import comm as dist
        self.global_rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        if topology is None:
            topology = PipeDataParallelTopology(1, self.world_size)
        self._topo = topology
        self.data_parallel_size = max(topology.get_dim("data"), 1)
        self.pipe_parallel_size = max(topology.get_dim("pipe"), 1)
        self.model_parallel_size = max(topology.get_dim("model"), 1)
        self.slice_parallel_size = self.model_parallel_size * self.pipe_parallel_size
        assert topology.world_size() == self.world_size, "topology size must equal world size"
        coord = topology.get_coord(self.global_rank)
        self.stage_id = coord.pipe if "pipe" in topology.axes else 0
        self.data_parallel_id = coord.data if "data" in topology.axes else 0
        self.model_parallel_id = coord.model if "model" in topology.axes else 0

        def mk(axis):
            mine = None
            for lst in topology.get_axis_comm_lists(axis):
                g = dist.new_group(lst)
                if self.global_rank in lst:
                    mine = (g, lst)
            return mine or (None, [self.global_rank])

        self.dp_group, self.dp_ranks = mk("data")
        self.pp_group, self.pp_ranks = mk("pipe")
        self.mp_group, self.mp_ranks = mk("model")
        # "slice" = every rank holding a different piece of the same model replica (pipe x model),
        # i.e. the ranks sharing this data-parallel coordinate (reference topology.py slice_proc_group)
        self.slice_group, self.slice_ranks = None, [self.global_rank]
        for d in range(self.data_parallel_size):
            lst = sorted(topology.filter_match(data=d)) if "data" in topology.axes else list(range(self.world_size))
            g = dist.new_group(lst)
            if self.global_rank in lst:
                self.slice_group, self.slice_ranks = g, lst
        self.ds_model_proc_group = self.mp_group
        # pipe-neighbour p2p groups are not needed: isend/irecv ride the world communicator.
        self.p2p_groups = None

    # Megatron-style accessors used by the engine
    def get_stage_id(self):
        return self.stage_id

    def get_data_parallel_id(self):
        return self.data_parallel_id

    def get_pipe_parallel_rank(self):
        return self.stage_id

    def get_pipe_parallel_world_size(self):
        return self.pipe_parallel_size

    def get_pipe_parallel_group(self):
        return self.pp_group

    def get_data_parallel_rank(self):
        return self.data_parallel_id

    def get_data_parallel_world_size(self):
        return self.data_parallel_size

    def get_data_parallel_group(self):
        return self.dp_group

    def get_model_parallel_rank(self):
        return self.model_parallel_id

    get_tensor_model_parallel_rank = get_model_parallel_rank

    def get_model_parallel_world_size(self):
        return self.model_parallel_size

    get_tensor_model_parallel_world_size = get_model_parallel_world_size

    def get_model_parallel_group(self):
        return self.mp_group

    get_tensor_model_parallel_group = get_model_parallel_group

    def get_slice_parallel_rank(self):
        return self.slice_ranks.index(self.global_rank)

    def get_slice_parallel_world_size(self):
        return self.slice_parallel_size

    def get_slice_parallel_group(self):
        return self.slice_group

    def stage_to_global(self, stage_id, **kwargs):
        me = self._topo.get_coord(self.global_rank)._asdict()
        me.update(kwargs)
        me["pipe"] = stage_id
        return self._topo.get_rank(**me)

    def topology(self):
        return self._topo

    def is_first_stage(self):
        return self.stage_id == 0

    def is_last_stage(self):
        return self.stage_id == self.pipe_parallel_size - 1
