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
