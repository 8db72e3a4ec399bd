"""Pipeline topologies and the per-rank grid view.

Reference parity: runtime/pipe/topology.py (``ProcessTopology`` :12, ``PipeDataParallelTopology``,
``PipeModelDataParallelTopology``, ``PipelineParallelGrid`` :250-456). The rank space and the groups
themselves live in utils/groups.py (one source of truth for DP/TP/PP/SP/EP); the grid is a thin view
answering "which stage am I, who are my neighbours, which group reduces my gradients".
"""
from ... import comm as dist
from ...utils import groups
from ...utils.groups import ProcessTopology  # noqa: F401  (re-export)


class PipeDataParallelTopology(ProcessTopology):

    def __init__(self, num_pp, num_dp):
        super().__init__(axes=["pipe", "data"], dims=[num_pp, num_dp])


class PipeModelDataParallelTopology(ProcessTopology):

    def __init__(self, num_pp, num_mp, num_dp):
        super().__init__(axes=["pipe", "data", "model"], dims=[num_pp, num_dp, num_mp])


class PipelineParallelGrid:
    """Stage / data / model coordinates of this rank inside the global ``groups`` topology."""

    def __init__(self, topology=None, process_group=None):
        self.global_rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        topo = groups.get_topology()
        self._topo = topo
        coord = topo.get_coord(self.global_rank)
        self.stage_id = coord["pipe"]
        self.data_parallel_id = coord["data"]
        self.model_parallel_id = coord["model"]
        self.seq_parallel_id = coord["seq"]
        self.pipe_parallel_size = topo.get_dim("pipe")
        self.data_parallel_size = topo.get_dim("data")
        self.model_parallel_size = topo.get_dim("model")
        self.slice_parallel_size = self.model_parallel_size
        self.pp_group = groups._get_group_ranks("pipe")
        self.dp_group = groups._get_group_ranks("data")
        self.pipe_group = groups._get_pipe_parallel_group()
        self.data_group = groups._get_data_parallel_group()

    def stage_to_global(self, stage_id, **kw):
        coord = self._topo.get_coord(self.global_rank)
        coord.update(pipe=stage_id, **kw)
        return self._topo.get_rank(**coord)

    def get_stage_id(self):
        return self.stage_id

    def get_data_parallel_id(self):
        return self.data_parallel_id

    def get_pipe_parallel_rank(self):
        return self.stage_id

    def get_pipe_parallel_world_size(self):
        return self.pipe_parallel_size

    def get_pipe_parallel_group(self):
        return self.pipe_group

    def get_data_parallel_rank(self):
        return self.data_parallel_id

    def get_data_parallel_world_size(self):
        return self.data_parallel_size

    def get_data_parallel_group(self):
        return self.data_group

    def get_model_parallel_rank(self):
        return self.model_parallel_id

    def get_model_parallel_world_size(self):
        return self.model_parallel_size

    def get_model_parallel_group(self):
        return groups._get_model_parallel_group()

    def get_slice_parallel_rank(self):
        return self.model_parallel_id

    def get_slice_parallel_world_size(self):
        return self.slice_parallel_size

    def is_first_stage(self):
        return self.stage_id == 0

    def is_last_stage(self):
        return self.stage_id == self.pipe_parallel_size - 1

    @property
    def prev_stage(self):
        return self.stage_id - 1

    @property
    def next_stage(self):
        return self.stage_id + 1
