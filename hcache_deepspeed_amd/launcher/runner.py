"""``hds`` / ``deepspeed`` launcher front-end: resource discovery, include/exclude filters, single-node
and multi-node dispatch.

Reference parity: launcher/runner.py (:48-631): hostfile ``host slots=N`` parsing, ``--include`` /
``--exclude`` NODE_SPEC[@NODE_SPEC] filters (``worker-0:0,1@worker-1``), ``--num_nodes`` /
``--num_gpus``, world info as urlsafe base64 JSON, single node -> ``python -m <pkg>.launcher.launch``,
multi node -> pdsh / OpenMPI / Slurm / MPICH / Intel MPI / MVAPICH command builders
(launcher/multinode_runner.py). Exported environment (``NCCL_*``, ``RCCL_*``, ``HSA_*``, ``HIP_*``,
``PYTHON*`` and ``.deepspeed_env`` entries) is forwarded to remote nodes.

MI355X specifics: local GPUs are counted from the KFD topology (no HIP initialisation in the launcher
process), device visibility uses ``HIP_VISIBLE_DEVICES``, and ``HSA_ENABLE_IPC_MODE_LEGACY=0`` (dmabuf
IPC, required by RCCL on this platform) is always forwarded.
"""
import argparse
import base64
import collections
import json
import os
import re
import shutil
import subprocess
import sys
from copy import deepcopy

from ..utils.logging import logger

DLTS_HOSTFILE = "/job/hostfile"
EXPORT_ENVS = ["MLFLOW", "NCCL", "RCCL", "HSA", "HIP", "ROCR", "ROCM", "PYTHON", "MV2", "UCX", "OMP", "TORCH",
               "PYTORCH", "HDS"]
DEEPSPEED_ENVIRONMENT_NAME = os.getenv("DS_ENV_FILE", ".deepspeed_env")
DEEPSPEED_ENVIRONMENT_PATHS = [os.path.expanduser("~"), "."]
PDSH_MAX_FAN_OUT = 1024
TORCH_DISTRIBUTED_DEFAULT_PORT = 29500


def parse_args(args=None):
    p = argparse.ArgumentParser(description="MI355X-native DeepSpeed-compatible launcher (one process per GPU).",
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("-H", "--hostfile", type=str, default=DLTS_HOSTFILE,
                   help="Hostfile: lines of '<hostname> slots=<gpus>'")
    p.add_argument("-i", "--include", type=str, default="", help="NODE_SPEC[@NODE_SPEC ...], NODE_SPEC=NAME[:SLOT[,SLOT]]")
    p.add_argument("-e", "--exclude", type=str, default="", help="Same syntax as --include; mutually exclusive")
    p.add_argument("--num_nodes", type=str, default="-1", help="Nodes to use (MIN:MAX with --elastic_training)")
    p.add_argument("--min_elastic_nodes", type=int, default=-1)
    p.add_argument("--max_elastic_nodes", type=int, default=-1)
    p.add_argument("--num_gpus", "--num_accelerators", type=int, default=-1, help="GPUs per node")
    p.add_argument("--master_port", default=TORCH_DISTRIBUTED_DEFAULT_PORT, type=int)
    p.add_argument("--master_addr", default="", type=str)
    p.add_argument("--node_rank", default=-1, type=int)
    p.add_argument("--launcher", default="pdsh", type=str,
                   help="Multi-node launcher: pdsh, openmpi, mpich, impi, slurm, mvapich")
    p.add_argument("--launcher_args", default="", type=str)
    p.add_argument("--module", action="store_true", help="Run user_script as 'python -m'")
    p.add_argument("--no_python", action="store_true", help="user_script is an executable, not a Python script")
    p.add_argument("--no_local_rank", action="store_true", help="Do not pass --local_rank to the user script")
    p.add_argument("--no_ssh", action="store_true", help="Launch each node independently (node_rank required)")
    p.add_argument("--no_ssh_check", action="store_true")
    p.add_argument("--force_multi", action="store_true", help="Use the multi-node path even on one node")
    p.add_argument("--save_pid", action="store_true")
    p.add_argument("--enable_each_rank_log", default="None", type=str)
    p.add_argument("--autotuning", default="", choices=["", "tune", "run"], type=str)
    p.add_argument("--elastic_training", action="store_true")
    p.add_argument("--bind_cores_to_rank", action="store_true", help="numactl-bind each rank to its core slice")
    p.add_argument("--bind_core_list", type=str, default=None)
    p.add_argument("--ssh_port", type=int, default=None)
    p.add_argument("user_script", type=str, help="User script (or module / executable)")
    p.add_argument("user_args", nargs=argparse.REMAINDER)
    return p.parse_args(args=args)


# ----------------------------------------------------------------------------------------
# hosts and resources
# ----------------------------------------------------------------------------------------
_HOST_LINE = re.compile(r"^(\S+)\s+slots=(\d+)\s*$")


def _parse_hostfile(lines):
    pool = collections.OrderedDict()
    for raw in lines:
        line = raw.split("#", 1)[0].strip()
        if not line:
            continue
        m = _HOST_LINE.match(line)
        if m is None:
            raise ValueError(f"Hostfile contains a bad entry: {raw.strip()!r}")
        host, slots = m.group(1), int(m.group(2))
        if host in pool:
            raise ValueError(f"Hostfile contains multiple entries for {host}")
        pool[host] = slots
    if not pool:
        raise ValueError("Hostfile is empty or not formatted correctly")
    return pool


def fetch_hostfile(path):
    if not os.path.isfile(path):
        logger.warning("no hostfile found, using local resources only")
        return None
    with open(path) as f:
        return _parse_hostfile(f.readlines())


def parse_node_config(spec):
    if ":" not in spec:
        return spec, []
    host, slots = spec.split(":", 1)
    return host, [int(s) for s in slots.split(",") if s != ""]


def parse_node_config_list(text):
    out = collections.OrderedDict()
    for spec in text.split("@"):
        if not spec:
            continue
        host, slots = parse_node_config(spec)
        out.setdefault(host, [])
        out[host] = sorted(set(out[host] + slots))
    return out


def parse_resource_filter(host_info, include_str="", exclude_str=""):
    """Apply an include OR exclude filter to {host: [slots]} (host order preserved)."""
    if include_str and exclude_str:
        raise ValueError("include_str and exclude_str are mutually exclusive.")
    if not include_str and not exclude_str:
        return host_info
    specs = parse_node_config_list(include_str or exclude_str)
    for host, slots in specs.items():
        if host not in host_info:
            raise ValueError(f"Hostname '{host}' not found in hostfile")
        for s in slots:
            if s not in host_info[host]:
                raise ValueError(f"No slot '{s}' specified on host '{host}'")
    if include_str:
        chosen = {h: (slots if slots else list(host_info[h])) for h, slots in specs.items()}
    else:
        chosen = deepcopy(dict(host_info))
        for h, slots in specs.items():
            chosen[h] = [s for s in chosen[h] if s not in slots] if slots else []
    out = collections.OrderedDict()
    for h in host_info:
        if h in chosen:
            uniq = list(dict.fromkeys(chosen[h]))
            if uniq:
                out[h] = uniq
    return out


def parse_inclusion_exclusion(resource_pool, inclusion, exclusion):
    active = collections.OrderedDict((h, list(range(n))) for h, n in resource_pool.items())
    return parse_resource_filter(active, include_str=inclusion, exclude_str=exclusion)


def encode_world_info(world_info):
    return base64.urlsafe_b64encode(json.dumps(world_info).encode("utf-8")).decode("utf-8")


def decode_world_info(b64):
    return json.loads(base64.urlsafe_b64decode(b64).decode("utf-8"))


def parse_num_nodes(text, elastic_training):
    parts = text.split(":")
    if len(parts) == 1:
        return int(parts[0]), -1
    if len(parts) == 2:
        if not elastic_training:
            raise RuntimeError("MIN:MAX format is only supported in elastic training")
        return int(parts[0]), int(parts[1])
    raise RuntimeError(f"num_nodes {text} is not in MIN:MAX format")


def local_gpu_count():
    """GPUs visible to this node without initialising HIP: KFD topology nodes with SIMDs."""
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        return len([v for v in vis.split(",") if v.strip() != ""])
    root = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "properties")) as f:
                    props = dict(line.split() for line in f if len(line.split()) == 2)
                if int(props.get("simd_count", "0")) > 0:
                    n += 1
            except OSError:
                continue
    except OSError:
        pass
    if n == 0:
        try:
            import torch
            n = torch.cuda.device_count()
        except Exception:  # noqa: BLE001
            n = 0
    return n


def _export_env(exports):
    env = {}
    for var, val in os.environ.items():
        if any(var.startswith(p) for p in EXPORT_ENVS):
            env[var] = val
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for d in DEEPSPEED_ENVIRONMENT_PATHS:
        path = os.path.join(d, DEEPSPEED_ENVIRONMENT_NAME)
        if os.path.isfile(path):
            with open(path) as f:
                for line in f:
                    line = line.strip()
                    if line and not line.startswith("#") and "=" in line:
                        k, v = line.split("=", 1)
                        env[k.strip()] = v.strip()
    env.update(exports)
    return env


# ----------------------------------------------------------------------------------------
def build_active_resources(args):
    pool = fetch_hostfile(args.hostfile)
    multi = pool is not None and (len(pool) > 1 or args.force_multi)
    if pool is None:
        n = args.num_gpus if args.num_gpus > 0 else local_gpu_count()
        if n <= 0:
            raise RuntimeError("no GPUs found on this node (set --num_gpus)")
        pool = collections.OrderedDict(localhost=n)
        if args.master_addr == "":
            args.master_addr = "127.0.0.1"
    active = parse_inclusion_exclusion(pool, args.include, args.exclude)
    min_nodes, _ = parse_num_nodes(args.num_nodes, args.elastic_training)
    if min_nodes > 0:
        active = collections.OrderedDict(list(active.items())[:min_nodes])
    if args.num_gpus > 0:
        active = collections.OrderedDict((h, s[:args.num_gpus]) for h, s in active.items())
    return active, multi


def build_local_cmd(args, world_info_b64):
    cmd = [sys.executable, "-u", "-m", "hcache_deepspeed_amd.launcher.launch", f"--world_info={world_info_b64}",
           f"--master_addr={args.master_addr or '127.0.0.1'}", f"--master_port={args.master_port}"]
    if args.node_rank >= 0:
        cmd.append(f"--node_rank={args.node_rank}")
    for flag in ("no_python", "no_local_rank", "module", "save_pid", "bind_cores_to_rank"):
        if getattr(args, flag):
            cmd.append(f"--{flag}")
    if args.bind_core_list:
        cmd.append(f"--bind_core_list={args.bind_core_list}")
    if args.enable_each_rank_log != "None":
        cmd.append(f"--enable_each_rank_log={args.enable_each_rank_log}")
    return cmd + [args.user_script] + list(args.user_args)


def main(args=None):
    args = parse_args(args)
    active, multi = build_active_resources(args)
    world_info = encode_world_info(active)
    if args.autotuning:
        from ..autotuning.autotuner import Autotuner
        tuner = Autotuner(args, active)
        tuner.tune()
        tuner.print_tuning_results()
        tuner.write_optimal_config()
        if args.autotuning == "run":
            tuner.run_after_tuning()
        return 0
    if not multi or args.no_ssh:
        cmd = build_local_cmd(args, world_info)
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    else:
        from .multinode_runner import RUNNERS
        if not args.master_addr:
            args.master_addr = list(active.keys())[0]
        runner_cls = RUNNERS.get(args.launcher.lower())
        if runner_cls is None:
            raise NotImplementedError(f"unknown launcher {args.launcher}")
        runner = runner_cls(args, world_info, active)
        if not runner.backend_exists():
            raise RuntimeError(f"launcher '{args.launcher}' not installed")
        env = _export_env({})
        cmd = runner.get_cmd(env, active)
        env = dict(os.environ, **runner.exports)
    logger.info(f"cmd = {' '.join(cmd)}")
    proc = subprocess.Popen(cmd, env=env)
    try:
        rc = proc.wait()
    except KeyboardInterrupt:
        proc.terminate()
        rc = proc.wait()
    if rc != 0:
        sys.exit(rc)
    return rc


def which(cmd):
    return shutil.which(cmd) is not None


if __name__ == "__main__":
    main()
