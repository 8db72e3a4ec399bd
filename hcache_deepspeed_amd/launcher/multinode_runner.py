"""Multi-node command builders: pdsh, OpenMPI, MPICH, Intel MPI, Slurm, MVAPICH.

Reference parity: launcher/multinode_runner.py (``PDSHRunner`` :55, ``OpenMPIRunner`` :124,
``MPICHRunner`` :204, ``IMPIRunner`` :276, ``SlurmRunner`` :361, ``MVAPICHRunner`` :409). pdsh starts
this package's per-node launcher on every host (``--node_rank=%n``); the MPI/Slurm runners start one
process per GPU directly and the ranks read their coordinates from the MPI/Slurm environment
(comm.init_distributed's discovery). RCCL-relevant variables are exported to every rank.
"""
import os
import shlex
import shutil
import sys


class MultiNodeRunner:
    name = "base"

    def __init__(self, args, world_info_base64, resource_pool=None):
        self.args = args
        self.world_info_base64 = world_info_base64
        self.resource_pool = resource_pool or {}
        self.user_script = args.user_script
        self.user_arguments = list(args.user_args)
        self.exports = {}
        self.validate_args()

    def backend_exists(self):
        return shutil.which(self.launcher_binary) is not None

    def add_export(self, key, var):
        self.exports[key.strip()] = str(var).strip()

    def validate_args(self):
        pass

    @property
    def world_size(self):
        return sum(len(v) if isinstance(v, (list, tuple)) else int(v) for v in self.resource_pool.values())

    @property
    def per_host(self):
        vals = list(self.resource_pool.values())
        return len(vals[0]) if vals and isinstance(vals[0], (list, tuple)) else (int(vals[0]) if vals else 0)

    def _python_cmd(self):
        if self.args.no_python:
            return [self.user_script]
        return [sys.executable, "-u"] + (["-m"] if self.args.module else []) + [self.user_script]

    def get_cmd(self, environment, active_resources):
        raise NotImplementedError


class PDSHRunner(MultiNodeRunner):
    name = "pdsh"
    launcher_binary = "pdsh"

    def get_cmd(self, environment, active_resources):
        environment["PDSH_RCMD_TYPE"] = "ssh"
        if self.args.ssh_port is not None:
            environment["PDSH_SSH_ARGS_APPEND"] = f"{environment.get('PDSH_SSH_ARGS_APPEND', '')} -p {self.args.ssh_port}"
        workers = ",".join(active_resources.keys())
        exports = "".join(f"export {k}={shlex.quote(str(v))}; " for k, v in {**environment, **self.exports}.items()
                          if k != "PDSH_RCMD_TYPE")
        launch = [exports + f"cd {os.path.abspath('.')};", sys.executable, "-u", "-m",
                  "hcache_deepspeed_amd.launcher.launch", f"--world_info={self.world_info_base64}", "--node_rank=%n",
                  f"--master_addr={self.args.master_addr}", f"--master_port={self.args.master_port}"]
        for flag in ("no_python", "module", "no_local_rank", "save_pid", "bind_cores_to_rank"):
            if getattr(self.args, flag, False):
                launch.append(f"--{flag}")
        if getattr(self.args, "bind_core_list", None):
            launch.append(f"--bind_core_list={self.args.bind_core_list}")
        user = [shlex.quote(a) for a in self.user_arguments]
        return ["pdsh", "-S", "-f", "1024", "-w", workers] + shlex.split(self.args.launcher_args) + launch + \
            [self.user_script] + user


class OpenMPIRunner(MultiNodeRunner):
    name = "openmpi"
    launcher_binary = "ompi_info"

    def validate_args(self):
        if self.args.include or self.args.exclude:
            raise ValueError(f"{self.name} backend does not support worker include/exclusion")
        if self.args.num_nodes != "-1" or self.args.num_gpus != -1:
            raise ValueError(f"{self.name} backend does not support limiting num nodes/gpus")

    def get_cmd(self, environment, active_resources):
        cmd = ["mpirun", "-n", str(self.world_size), "-hostfile", self.args.hostfile, "--mca", "btl", "^openib",
               "--mca", "btl_tcp_if_include", "eth0"] + shlex.split(self.args.launcher_args)
        for k, v in {**self.exports, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}.items():
            cmd += ["-x", f"{k}={v}"]
        return cmd + self._python_cmd() + self.user_arguments


class MPICHRunner(MultiNodeRunner):
    name = "mpich"
    launcher_binary = "hydra_pmi_proxy"

    def get_cmd(self, environment, active_resources):
        hosts = ",".join(f"{h}:{len(s) if isinstance(s, (list, tuple)) else s}" for h, s in active_resources.items())
        cmd = ["mpirun", "-n", str(self.world_size), "-ppn", str(self.per_host), "-hosts", hosts] + \
            shlex.split(self.args.launcher_args)
        for k, v in {**self.exports, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}.items():
            cmd += ["-genv", k, str(v)]
        return cmd + self._python_cmd() + self.user_arguments


class IMPIRunner(MPICHRunner):
    name = "impi"
    launcher_binary = "mpiexec.hydra"


class SlurmRunner(MultiNodeRunner):
    name = "slurm"
    launcher_binary = "srun"

    def get_cmd(self, environment, active_resources):
        cmd = ["srun", "-n", str(self.world_size)] + shlex.split(self.args.launcher_args)
        if self.args.include:
            cmd.append(f"--nodelist={self.args.include}")
        if self.args.exclude:
            cmd.append(f"--exclude={self.args.exclude}")
        if self.args.num_nodes != "-1":
            cmd.append(f"--nodes={self.args.num_nodes}")
        if self.args.num_gpus > 0:
            cmd.append(f"--gpus={self.args.num_gpus}")
        exports = ",".join(f"{k}={v}" for k, v in {**self.exports, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}.items())
        cmd.append(f"--export=ALL,{exports}")
        return cmd + self._python_cmd() + self.user_arguments


class MVAPICHRunner(MultiNodeRunner):
    name = "mvapich"
    launcher_binary = "mpiname"

    def __init__(self, args, world_info_base64, resource_pool=None):
        super().__init__(args, world_info_base64, resource_pool)
        self.add_export("MV2_SMP_USE_CMA", "0")
        self.add_export("MV2_DEBUG_SHOW_BACKTRACE", "1")
        self.add_export("MV2_SUPPORT_DL", "1")
        self.add_export("MV2_ENABLE_AFFINITY", "0")

    def get_cmd(self, environment, active_resources):
        hostfile = "/tmp/hds_mvapich_hostfile"
        with open(hostfile, "w") as f:
            for h in active_resources:
                f.write(f"{h}\n")
        cmd = ["mpirun", "-np", str(self.world_size), "-ppn", str(self.per_host), "--hostfile", hostfile] + \
            shlex.split(self.args.launcher_args)
        for k, v in {**self.exports, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}.items():
            cmd += ["-env", f"{k}={v}"]
        return cmd + self._python_cmd() + self.user_arguments


RUNNERS = {r.name: r for r in (PDSHRunner, OpenMPIRunner, MPICHRunner, IMPIRunner, SlurmRunner, MVAPICHRunner)}
