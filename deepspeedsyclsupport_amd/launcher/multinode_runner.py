"""Multi-node runners (reference `launcher/multinode_runner.py:51-458`): build the command that starts
`launcher.launch` on every node (pdsh) or every rank directly (MPI flavours, Slurm)."""
import os
import shutil
import sys
from abc import ABC, abstractmethod

from .constants import MVAPICH_TMP_HOSTFILE, PDSH_MAX_FAN_OUT


class MultiNodeRunner(ABC):

    def __init__(self, args, world_info_base64, resources=None):
        self.args = args
        self.world_info_base64 = world_info_base64
        self.resources = resources or {}
        self.exports = {}
        self.user_arguments = self.parse_user_args()
        self.user_script = args.user_script

    def add_export(self, key, var):
        self.exports[key.strip()] = str(var).strip()

    def parse_user_args(self):
        return list(self.args.user_args)

    @property
    def name(self):
        return self.__class__.__name__

    @abstractmethod
    def backend_exists(self):
        ...

    @abstractmethod
    def get_cmd(self, environment, active_resources):
        ...

    def _world_size(self, active):
        return sum(len(s) for s in active.values())

    def _python_cmd(self):
        cmd = [] if self.args.no_python else [sys.executable, "-u"] + (["-m"] if self.args.module else [])
        return cmd + [self.user_script] + self.user_arguments


class PDSHRunner(MultiNodeRunner):

    def backend_exists(self):
        return shutil.which("pdsh") is not None

    def get_cmd(self, environment, active_resources):
        environment["PDSH_RCMD_TYPE"] = "ssh"
        if self.args.ssh_port is not None:
            environment["PDSH_SSH_ARGS_APPEND"] = f"-p {self.args.ssh_port}"
        hosts = ",".join(active_resources.keys())
        exports = "".join(f"export {k}={v}; " for k, v in self.exports.items())
        launch = [exports, f"cd {os.path.abspath('.')};", sys.executable, "-u", "-m",
                  "deepspeedsyclsupport_amd.launcher.launch", f"--world_info={self.world_info_base64}",
                  "--node_rank=%n", f"--master_addr={self.args.master_addr}",
                  f"--master_port={self.args.master_port}"]
        for flag in ("no_python", "no_local_rank", "module"):
            if getattr(self.args, flag):
                launch.append(f"--{flag}")
        return (["pdsh", "-S", "-f", str(PDSH_MAX_FAN_OUT), "-w", hosts] + self.args.launcher_args.split() + launch +
                [self.user_script] + self.user_arguments)


class OpenMPIRunner(MultiNodeRunner):

    def backend_exists(self):
        return shutil.which("ompi_info") is not None

    def get_cmd(self, environment, active_resources):
        total = self._world_size(active_resources)
        hosts = ",".join(f"{h}:{len(s)}" for h, s in active_resources.items())
        cmd = ["mpirun", "-n", str(total), "-host", hosts, "--mca", "btl", "^openib", "--mca", "btl_tcp_if_include",
               "eth0"] + self.args.launcher_args.split()
        for k, v in self.exports.items():
            cmd += ["-x", f"{k}={v}"]
        return cmd + self._python_cmd()


class MPICHRunner(MultiNodeRunner):

    def backend_exists(self):
        return shutil.which("mpirun") is not None and shutil.which("ompi_info") is None

    def get_cmd(self, environment, active_resources):
        total = self._world_size(active_resources)
        per_node = len(next(iter(active_resources.values())))
        cmd = ["mpirun", "-n", str(total), "-ppn", str(per_node), "-hosts", ",".join(active_resources)]
        for k, v in self.exports.items():
            cmd += ["-genv", k, v]
        return cmd + self.args.launcher_args.split() + self._python_cmd()


class IMPIRunner(MPICHRunner):

    def backend_exists(self):
        return shutil.which("mpirun") is not None and "I_MPI_ROOT" in os.environ


class SlurmRunner(MultiNodeRunner):

    def backend_exists(self):
        return shutil.which("sinfo") is not None

    def get_cmd(self, environment, active_resources):
        total = self._world_size(active_resources)
        cmd = ["srun", "-n", str(total)] + self.args.launcher_args.split()
        if self.args.include:
            cmd += ["--include", self.args.include]
        if self.args.exclude:
            cmd += ["--exclude", self.args.exclude]
        if self.args.num_nodes > 0:
            cmd += ["--nodes", str(self.args.num_nodes)]
        exports = ",".join(f"{k}={v}" for k, v in self.exports.items())
        cmd += [f"--export=ALL{',' + exports if exports else ''}"]
        return cmd + self._python_cmd()


class MVAPICHRunner(MultiNodeRunner):

    def backend_exists(self):
        return shutil.which("mpiname") is not None

    def get_cmd(self, environment, active_resources):
        total = self._world_size(active_resources)
        per_node = len(next(iter(active_resources.values())))
        with open(MVAPICH_TMP_HOSTFILE, "w") as f:
            for h in active_resources:
                f.write(f"{h}\n")
        cmd = ["mpirun", "-np", str(total), "-ppn", str(per_node), "--hostfile", MVAPICH_TMP_HOSTFILE]
        for k, v in self.exports.items():
            cmd += ["-env", f"{k}={v}"]
        return cmd + self.args.launcher_args.split() + self._python_cmd()


RUNNERS = {"pdsh": PDSHRunner, "openmpi": OpenMPIRunner, "mpich": MPICHRunner, "impi": IMPIRunner,
           "slurm": SlurmRunner, "mvapich": MVAPICHRunner}
