"""Elastic worker agent: restarts the node's worker group on failure or membership change.

Reference parity: elasticity/elastic_agent.py ``DSElasticAgent`` (:32-190): a torch-elastic
``LocalElasticAgent`` whose workers get the DeepSpeed env (MASTER_*, RANK, LOCAL_RANK, WORLD_SIZE,
CROSS_*), restarted up to ``max_restarts`` times when the group turns UNHEALTHY/FAILED or the
rendezvous membership changes. MI355X: RCCL error handling and dmabuf IPC are forced on for workers.
"""
import os

from ..utils.logging import logger

try:
    from torch.distributed.elastic.agent.server.local_elastic_agent import LocalElasticAgent
    _HAVE_ELASTIC = True
except ImportError:  # pragma: no cover
    LocalElasticAgent = object
    _HAVE_ELASTIC = False


class DSElasticAgent(LocalElasticAgent):

    def __init__(self, spec, env, start_method="spawn", exit_barrier_timeout=300, log_line_prefix_template=None):
        if not _HAVE_ELASTIC:
            raise RuntimeError("torch.distributed.elastic is not available")
        super().__init__(spec, start_method=start_method, exit_barrier_timeout=exit_barrier_timeout)
        self.ds_env = dict(env)
        self.ds_env.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        self.ds_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

    def _start_workers(self, worker_group):
        # expose the agent-level environment to every (re)started worker
        for k, v in self.ds_env.items():
            os.environ.setdefault(k, v)
        return super()._start_workers(worker_group)


def run_elastic(cmd, env, n_local, args):
    """Run ``cmd`` as ``n_local`` elastic workers under a c10d rendezvous (launch.py --enable_elastic_training)."""
    from torch.distributed.elastic.agent.server.api import WorkerSpec
    from torch.distributed.elastic.rendezvous import RendezvousParameters
    import torch.distributed.elastic.rendezvous.registry as rdzv_registry
    min_nodes = args.min_elastic_nodes if args.min_elastic_nodes > 0 else 1
    max_nodes = args.max_elastic_nodes if args.max_elastic_nodes > 0 else int(env.get("CROSS_SIZE", "1"))
    params = RendezvousParameters(backend="c10d", endpoint=f"{args.master_addr}:{args.master_port}",
                                  run_id=os.environ.get("ELASTIC_RUN_ID", "hds-elastic"), min_nodes=min_nodes,
                                  max_nodes=max_nodes, timeout=100)
    spec = WorkerSpec(role="trainer", local_world_size=n_local, entrypoint=cmd[0], args=tuple(cmd[1:]),
                      rdzv_handler=rdzv_registry.get_rendezvous_handler(params), max_restarts=100,
                      monitor_interval=5)
    agent = DSElasticAgent(spec, env)
    result = agent.run()
    logger.info(f"elastic run finished: {result.state}")
    return 0 if not result.is_failed() else 1
