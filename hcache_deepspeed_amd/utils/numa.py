"""numactl core binding per rank (reference utils/numa.py:24-205: ``get_numa_cores``, ``parse_range_list``,
``get_numactl_cmd``). Core slices are taken from the NUMA node of the rank's GPU when sysfs exposes it (MI355X
nodes: 4 GPUs per socket), otherwise from the whole core list split evenly across local ranks."""
import os
import shutil


def parse_range(rng):
    if "-" in rng:
        lo, hi = rng.split("-", 1)
        lo, hi = int(lo), int(hi)
        if lo > hi:
            raise ValueError(f"bad range {rng}")
        return list(range(lo, hi + 1))
    return [int(rng)]


def parse_range_list(text):
    """'0,2-4,7' -> [0, 2, 3, 4, 7] (sorted, unique)."""
    out = []
    for part in text.split(","):
        part = part.strip()
        if part:
            out += parse_range(part)
    if sorted(set(out)) != out:
        raise ValueError(f"core list {text} must be sorted and unique")
    return out


def get_numa_cores():
    """[[cores of NUMA node 0], [cores of node 1], ...] from sysfs."""
    root = "/sys/devices/system/node"
    nodes = []
    if os.path.isdir(root):
        for d in sorted(os.listdir(root)):
            if d.startswith("node") and d[4:].isdigit():
                try:
                    with open(os.path.join(root, d, "cpulist")) as f:
                        nodes.append(parse_range_list(f.read().strip()))
                except (OSError, ValueError):
                    continue
    return nodes


def get_numactl_cmd(bind_core_list, num_local_procs, local_rank):
    """Returns (cores_per_rank, ['numactl', '-C', '<cores>', ...])."""
    if bind_core_list:
        cores = parse_range_list(bind_core_list)
    else:
        cores = list(range(os.cpu_count() or 1))
    per = max(1, len(cores) // num_local_procs)
    mine = cores[local_rank * per:(local_rank + 1) * per]
    cmd = []
    if shutil.which("numactl"):
        cmd = ["numactl", "-C", ",".join(str(c) for c in mine)]
        numa = get_numa_cores()
        for node, ncores in enumerate(numa):
            if set(mine) <= set(ncores):
                cmd += ["-m", str(node)]
                break
    return per, cmd


# ---------------------------------------------------------------------------------------------------------------
# per-rank host threads (reference launcher/launch.py:230-233 sets OMP_NUM_THREADS to the rank's core slice when it
# binds cores; under torch.distributed.run nothing does, and torchrun forces OMP_NUM_THREADS=1 for nproc > 1)
# ---------------------------------------------------------------------------------------------------------------
def _cgroup_cpu_budget():
    """CPUs the cgroup quota allows (cgroup v2 ``cpu.max``, v1 ``cfs_quota_us``), or None when unlimited."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                text = f.read().strip()
        except OSError:
            continue
        if parse is not None:
            q, p = parse(text)[:2]
            if q == "max":
                return None
            return max(1, int(int(q) / int(p)))
        q = int(text)
        if q <= 0:
            return None
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                return max(1, int(q / int(f.read().strip())))
        except OSError:
            return None
    return None


def rank_core_slice(local_rank, local_world, cpus=None, numa=None, budget=None):
    """The cores of local rank ``local_rank`` of ``local_world``: ranks are dealt to the NUMA nodes in order (GPUs
    0..k-1 sit on socket 0 on MI355X nodes) and each node's usable cores are split evenly among its ranks; without
    NUMA information the usable cores are split evenly. ``budget`` (cgroup quota) caps the cores per rank."""
    cpus = sorted(cpus if cpus is not None else (os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity")
                                                 else range(os.cpu_count() or 1)))
    numa = [sorted(set(n) & set(cpus)) for n in (numa if numa is not None else get_numa_cores())]
    numa = [n for n in numa if n]
    if len(numa) > 1 and local_world >= len(numa):
        node = local_rank * len(numa) // local_world
        ranks_on = [r for r in range(local_world) if r * len(numa) // local_world == node]
        pool, k, idx = numa[node], len(ranks_on), ranks_on.index(local_rank)
    else:
        pool, k, idx = cpus, local_world, local_rank
    per = max(1, len(pool) // k)
    if budget:
        per = max(1, min(per, budget // local_world))
    mine = pool[idx * per:(idx + 1) * per] or pool[:per]
    return mine


def configure_rank_threads(setting="auto", local_rank=None, local_world=None, bind=None):
    """Give this rank its share of the host's CPUs for the C++ host kernels (``hds_cpu_set_num_threads``) and torch's
    CPU ops (``torch.set_num_threads``); with ``bind`` (default: only when nothing bound the process yet, and not with
    HDS_BIND_CORES=0) also pin the process to that NUMA-local slice. ``setting``: "auto" or an int. Returns the record
    reported in the bench JSON ``extra.host_threads``."""
    import torch
    global _configured
    key = (str(setting), local_rank, local_world, bind)
    if _configured is not None and _configured[0] == key:
        return dict(_configured[1])  # once per process: a second engine must not slice the slice again
    local_world = int(local_world if local_world is not None else os.environ.get("LOCAL_WORLD_SIZE", "1"))
    local_rank = int(local_rank if local_rank is not None else os.environ.get("LOCAL_RANK", "0"))
    rec = {"local_world": local_world, "source": "default"}
    explicit = os.environ.get("HDS_CPU_THREADS")
    if setting not in (None, "auto", "AUTO"):
        explicit = setting
    n, cores = None, None
    if explicit is not None and str(explicit).strip():
        n, rec["source"] = max(1, int(explicit)), "explicit"
    elif local_world > 1 and os.environ.get("OMP_NUM_THREADS", "1") == "1":
        # several ranks on one host and nobody chose a count (torchrun's forced 1 or unset): the rank's slice
        have = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
        cores = rank_core_slice(local_rank, local_world, cpus=have, budget=_cgroup_cpu_budget())
        n, rec["source"] = len(cores), "auto"
        allcpu = set(range(os.cpu_count() or 1))
        if bind is None:
            bind = os.environ.get("HDS_BIND_CORES", "1") != "0" and set(have) == allcpu and len(cores) < len(have)
        if bind and hasattr(os, "sched_setaffinity"):
            try:
                os.sched_setaffinity(0, cores)
                rec["bound"] = True
            except OSError:
                rec["bound"] = False
        rec["cores"] = f"{cores[0]}-{cores[-1]}" if cores else ""
    if n is not None:
        torch.set_num_threads(n)
        try:
            from ..ops import native
            lib = native.host_lib()
            if lib is not None:
                lib.hds_cpu_set_num_threads(n)
        except Exception:  # noqa: BLE001 -- host library absent (pure-python CPU runs): torch's count still applies
            pass
    rec["threads"] = n if n is not None else torch.get_num_threads()
    try:
        from ..ops import native
        lib = native.host_lib()
        if lib is not None:
            rec["host_kernel_threads"] = int(lib.hds_cpu_num_threads())
    except Exception:  # noqa: BLE001
        pass
    _configured = (key, dict(rec))
    return rec


_configured = None
