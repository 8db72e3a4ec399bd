"""Process-group topology: DP / TP / PP / SP / EP groups on one flat rank space.

Reference parity: deepspeed/utils/groups.py (``_get_data_parallel_group`` :519,
``_get_sequence_parallel_group`` :611, ``_get_expert_parallel_group`` :451,
``_create_expert_and_data_parallel``, ``_create_zero_param_parallel_group`` :650) and
runtime/pipe/topology.py (``ProcessTopology``).

Rank layout (fastest-varying last): ``rank = ((pp * DP + dp) * SP + sp) * TP + tp``. Tensor
parallelism gets adjacent ranks: on one 8x MI355X node every pair of GPUs has its own xGMI link,
so adjacency does not matter for bandwidth, but it keeps TP inside one node when scaling out.
Expert parallel groups are carved out of the (dp x sp) "expert-data" space, E+D layout.
"""
import itertools

from .. import comm as dist


class ProcessTopology:
    """Cartesian rank topology with named axes (reference: runtime/pipe/topology.py:12)."""

    def __init__(self, axes, dims):
        self.axes = list(axes)
        self.dims = list(dims)
        self.mapping = {}
        for rank, coord in enumerate(itertools.product(*[range(d) for d in self.dims])):
            self.mapping[coord] = rank

    def world_size(self):
        n = 1
        for d in self.dims:
            n *= d
        return n

    def get_rank(self, **coords):
        key = tuple(coords[a] for a in self.axes)
        return self.mapping[key]

    def get_coord(self, rank):
        for c, r in self.mapping.items():
            if r == rank:
                return dict(zip(self.axes, c))
        raise ValueError(rank)

    def get_dim(self, axis):
        return self.dims[self.axes.index(axis)]

    def get_axis_comm_lists(self, axis):
        """All rank lists that vary only along ``axis``."""
        idx = self.axes.index(axis)
        others = [range(d) for i, d in enumerate(self.dims) if i != idx]
        lists = []
        for oc in itertools.product(*others):
            ranks = []
            for k in range(self.dims[idx]):
                c = list(oc)
                c.insert(idx, k)
                ranks.append(self.mapping[tuple(c)])
            lists.append(ranks)
        return lists

    def filter_match(self, **filt):
        return [r for c, r in self.mapping.items() if all(c[self.axes.index(k)] == v for k, v in filt.items())]


class PipeModelDataParallelTopology(ProcessTopology):

    def __init__(self, num_pp, num_mp, num_dp):
        super().__init__(axes=["pipe", "data", "model"], dims=[num_pp, num_dp, num_mp])


class _State:
    topo = None
    groups = {}
    rank_lists = {}
    expert_groups = {}
    expert_data_groups = {}


def _make(axis_lists, name):
    me = dist.get_rank()
    mine = None
    for ranks in axis_lists:
        g = dist.new_group(ranks=ranks) if dist.is_initialized() and dist.get_world_size() > 1 else None
        if me in ranks:
            mine = g
            _State.rank_lists[name] = ranks
    _State.groups[name] = mine
    return mine


def initialize(tp=1, pp=1, sp=1, ep=1, dp=None):
    """Build all groups. ``dp`` defaults to world // (tp*pp*sp). Must be called on every rank."""
    world = dist.get_world_size()
    if dp is None:
        assert world % (tp * pp * sp) == 0, f"world {world} not divisible by tp*pp*sp={tp * pp * sp}"
        dp = world // (tp * pp * sp)
    assert dp * tp * pp * sp == world
    topo = ProcessTopology(["pipe", "data", "seq", "model"], [pp, dp, sp, tp])
    _State.topo = topo
    _State.groups, _State.rank_lists = {}, {}
    _make(topo.get_axis_comm_lists("data"), "data")
    _make(topo.get_axis_comm_lists("model"), "model")
    _make(topo.get_axis_comm_lists("pipe"), "pipe")
    _make(topo.get_axis_comm_lists("seq"), "seq")
    # sequence-data-parallel: ranks sharing (pipe, model) coords -> ZeRO shards over dp x sp
    sdp = {}
    for c, r in topo.mapping.items():
        key = (c[0], c[3])
        sdp.setdefault(key, []).append(r)
    _make(list(sdp.values()), "seq_data")
    # expert parallel inside the seq_data space (E+D: consecutive ranks form an EP group)
    if ep > 1:
        _create_expert_and_data_parallel(ep)
    return topo


def _create_expert_and_data_parallel(ep_size, name=None):
    name = name or f"ep_size_{ep_size}"
    base = _State.rank_lists.get("seq_data") or list(range(dist.get_world_size()))
    spaces = [base]
    if _State.topo is not None:
        spaces = []
        seen = set()
        for c, r in _State.topo.mapping.items():
            key = (c[0], c[3])
            if key in seen:
                continue
            seen.add(key)
            spaces.append(sorted(rr for cc, rr in _State.topo.mapping.items() if (cc[0], cc[3]) == key))
    me = dist.get_rank()
    for space in spaces:
        n = len(space)
        assert n % ep_size == 0, f"expert parallel size {ep_size} must divide data-parallel size {n}"
        for i in range(n // ep_size):
            ranks = space[i * ep_size:(i + 1) * ep_size]
            g = dist.new_group(ranks=ranks) if dist.get_world_size() > 1 else None
            if me in ranks:
                _State.expert_groups[name] = g
                _State.rank_lists["ep:" + name] = ranks
        for j in range(ep_size):
            ranks = space[j::ep_size]
            g = dist.new_group(ranks=ranks) if dist.get_world_size() > 1 else None
            if me in ranks:
                _State.expert_data_groups[name] = g
                _State.rank_lists["edp:" + name] = ranks
    return name


def _ensure():
    if _State.topo is None:
        initialize()


def _get(name):
    _ensure()
    return _State.groups.get(name)


def _get_data_parallel_group():
    return _get("data")


def _get_model_parallel_group():
    return _get("model")


def _get_pipe_parallel_group():
    return _get("pipe")


def _get_sequence_parallel_group():
    return _get("seq")


def _get_sequence_data_parallel_group():
    return _get("seq_data")


def _get_expert_parallel_group(group_name):
    return _State.expert_groups[group_name]


def _get_expert_data_parallel_group(group_name):
    return _State.expert_data_groups[group_name]


def expert_data_group_of(p):
    """Expert-data-parallel group of an MoE parameter; ``False`` for dense params (or EP not set up)."""
    if getattr(p, "allreduce", True):
        return False
    name = getattr(p, "group_name", None)
    if name is None or name not in _State.expert_data_groups:
        return False
    return _State.expert_data_groups[name]


def _get_expert_parallel_group_dict():
    return dict(_State.expert_groups)


def _get_group_ranks(name):
    _ensure()
    return _State.rank_lists.get(name, [dist.get_rank()])


def _size(name):
    _ensure()
    return len(_State.rank_lists.get(name, [0]))


def get_data_parallel_world_size():
    return _size("data")


def get_model_parallel_world_size():
    return _size("model")


def get_tensor_model_parallel_world_size():
    return _size("model")


def get_pipe_parallel_world_size():
    return _size("pipe")


def get_sequence_parallel_world_size():
    return _size("seq")


def get_sequence_data_parallel_world_size():
    return _size("seq_data")


def _rank_in(name):
    _ensure()
    ranks = _State.rank_lists.get(name, [dist.get_rank()])
    return ranks.index(dist.get_rank())


def get_data_parallel_rank():
    return _rank_in("data")


def get_model_parallel_rank():
    return _rank_in("model")


def get_tensor_model_parallel_rank():
    return _rank_in("model")


def get_sequence_parallel_rank():
    return _rank_in("seq")


def get_sequence_data_parallel_rank():
    return _rank_in("seq_data")


def get_topology():
    _ensure()
    return _State.topo


def reset():
    _State.topo = None
    _State.groups, _State.rank_lists = {}, {}
    _State.expert_groups, _State.expert_data_groups = {}, {}
