"""Per-node launcher: one process per local MI355X, rendezvous env, failure propagation.

Reference parity: launcher/launch.py (:133-359): decodes the world info, computes global ranks in host
order, exports MASTER_ADDR/PORT, WORLD_SIZE, RANK, LOCAL_RANK, LOCAL_SIZE, CROSS_RANK, CROSS_SIZE,
restricts device visibility, optionally pins each rank with numactl, forwards SIGINT/SIGTERM to the
children and tears the whole tree down on the first non-zero exit; ``--enable_elastic_training`` runs
the workers under :class:`~hcache_deepspeed_amd.elasticity.elastic_agent.DSElasticAgent`.

MI355X: ranks see ALL local GPUs (``HIP_VISIBLE_DEVICES`` = the node's slot list) and select theirs with
``LOCAL_RANK``, which keeps RCCL's xGMI peer discovery intact; the CPU binding uses the GPU's NUMA node
from sysfs when ``--bind_cores_to_rank`` is given without an explicit core list.
"""
import argparse
import os
import signal
import subprocess
import sys
import time

from ..utils.logging import logger
from .runner import decode_world_info

PID_FILE_BASEPATH = "/tmp"


def parse_args(args=None):
    p = argparse.ArgumentParser(description="per-node process launcher")
    p.add_argument("--node_rank", type=int, default=0)
    p.add_argument("--master_addr", default="127.0.0.1", type=str)
    p.add_argument("--master_port", default=29500, type=int)
    p.add_argument("--world_info", default="None", type=str)
    p.add_argument("--module", action="store_true")
    p.add_argument("--no_python", action="store_true")
    p.add_argument("--enable_elastic_training", action="store_true")
    p.add_argument("--min_elastic_nodes", type=int, default=-1)
    p.add_argument("--max_elastic_nodes", type=int, default=-1)
    p.add_argument("--no_local_rank", action="store_true")
    p.add_argument("--save_pid", action="store_true")
    p.add_argument("--enable_each_rank_log", default="None", type=str)
    p.add_argument("--bind_cores_to_rank", action="store_true")
    p.add_argument("--bind_core_list", type=str, default=None)
    p.add_argument("training_script", type=str)
    p.add_argument("training_script_args", nargs=argparse.REMAINDER)
    return p.parse_args(args=args)


def rank_mapping(world_info):
    """{host: [global ranks]} in host order, and the world size."""
    mapping, r = {}, 0
    for host, slots in world_info.items():
        mapping[host] = list(range(r, r + len(slots)))
        r += len(slots)
    return mapping, r


def build_env(base_env, world_info, node_rank, master_addr, master_port):
    hosts = list(world_info.keys())
    local = hosts[node_rank]
    mapping, world = rank_mapping(world_info)
    env = dict(base_env)
    env.update(MASTER_ADDR=master_addr, MASTER_PORT=str(master_port), WORLD_SIZE=str(world),
               CROSS_RANK=str(node_rank), CROSS_SIZE=str(len(hosts)), LOCAL_SIZE=str(len(world_info[local])))
    env["HIP_VISIBLE_DEVICES"] = ",".join(str(s) for s in world_info[local])
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("DEBUG_CLR_LIMIT_BLIT_WG", "16")  # before the rank loads HIP (hcache_deepspeed_amd/__init__.py)
    return env, mapping[local]


def build_rank_cmd(args, local_rank, n_local):
    cmd, extra_env = [], {}
    if args.bind_cores_to_rank:
        from ..utils.numa import get_numactl_cmd
        cores, numactl = get_numactl_cmd(args.bind_core_list, n_local, local_rank)
        extra_env["OMP_NUM_THREADS"] = str(cores)
        cmd += numactl
    if not args.no_python:
        cmd += [sys.executable, "-u"]
        if args.module:
            cmd.append("-m")
    elif args.module:
        raise ValueError("--no_python and --module are mutually exclusive")
    cmd.append(args.training_script)
    if not args.no_local_rank:
        cmd.append(f"--local_rank={local_rank}")
    return cmd + list(args.training_script_args), extra_env


def _terminate(procs):
    for p in procs:
        if p.poll() is None:
            try:
                p.terminate()
            except OSError:
                pass
    deadline = time.time() + 30
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()


def main(args=None):
    args = parse_args(args)
    if args.world_info == "None":
        raise ValueError("world_info can not be None")
    world_info = decode_world_info(args.world_info)
    env, ranks = build_env(os.environ, world_info, args.node_rank, args.master_addr, args.master_port)
    n_local = len(ranks)
    logger.info(f"node {args.node_rank}: ranks {ranks}, world {env['WORLD_SIZE']}")
    pid_file = None
    if args.save_pid:
        pid_file = os.path.join(PID_FILE_BASEPATH, f"{os.getpid()}.deepspeed")
        with open(pid_file, "w") as f:
            f.write(str(os.getpid()))

    if args.enable_elastic_training:
        from ..elasticity.elastic_agent import run_elastic
        cmd, _ = build_rank_cmd(args, 0, n_local)
        cmd = [c for c in cmd if not c.startswith("--local_rank=")]
        return run_elastic(cmd, env, n_local, args)

    log_dir = None if args.enable_each_rank_log == "None" else args.enable_each_rank_log
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
    stamp = time.strftime("%Y%m%d%H%M%S")
    procs, logs = [], []
    for local_rank, rank in enumerate(ranks):
        renv = dict(env, RANK=str(rank), LOCAL_RANK=str(local_rank))
        cmd, extra = build_rank_cmd(args, local_rank, n_local)
        renv.update(extra)
        out = None
        if log_dir:
            out = open(os.path.join(log_dir, f"{stamp}_rank{rank}.log"), "w")
            logs.append(out)
        procs.append(subprocess.Popen(cmd, env=renv, stdout=out, stderr=out))
        logger.info(f"rank {rank} (pid {procs[-1].pid}): {' '.join(cmd)}")

    state = {"rc": None}

    def on_signal(signum, frame):
        _terminate(procs)
        if pid_file and os.path.isfile(pid_file):
            os.remove(pid_file)
        sys.exit(state["rc"] if state["rc"] else 1)

    signal.signal(signal.SIGINT, on_signal)
    signal.signal(signal.SIGTERM, on_signal)
    alive = list(procs)
    while alive:
        for p in list(alive):
            rc = p.poll()
            if rc is None:
                continue
            alive.remove(p)
            if rc != 0:
                state["rc"] = rc
                logger.error(f"process {p.pid} exited with {rc}; terminating the node's other ranks")
                _terminate(alive)
                alive = []
                break
        time.sleep(0.2)
    for f in logs:
        f.close()
    if pid_file and os.path.isfile(pid_file):
        os.remove(pid_file)
    if state["rc"]:
        sys.exit(state["rc"])
    return 0


if __name__ == "__main__":
    main()
